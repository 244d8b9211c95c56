"""N>1 path of bench.py on CPU: two gloo ranks on 127.0.0.1 (the GPU path uses the same
helpers over RCCL). Replicas design: one weight broadcast at load, disjoint
utterance seeds per rank, max-over-ranks wall time; no per-step collective.
"""

import hashlib
import multiprocessing as mp
import os
import socket
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world))
        sys.path.insert(0, str(ROOT))
        sys.path.insert(0, str(ROOT / "pocket-tts_amd"))
        import numpy as np
        import torch
        import torch.distributed as dist

        import bench
        import pocket_tts_amd as pt

        dist.init_process_group("gloo", rank=rank, world_size=world)
        n = pt.Engine.weight_blob_bytes() // 4
        if rank == 0:
            blob = torch.from_numpy(pt.Engine.pack_weights(0x5EED))
        else:
            blob = torch.full((n,), float("nan"), dtype=torch.float32)
        bench.broadcast_weights(dist, blob)
        got = hashlib.sha256(blob.numpy().tobytes()).hexdigest()
        # every rank could have packed the same blob itself: the broadcast must reproduce it
        own = hashlib.sha256(pt.Engine.pack_weights(0x5EED).tobytes()).hexdigest()
        times = bench.max_over_ranks(dist, [1.0 + rank, 10.0 - rank], "cpu")
        seeds = torch.tensor([bench.slot_seed(1, rank, b) for b in range(32)], dtype=torch.int64)
        all_seeds = [torch.empty_like(seeds) for _ in range(world)]
        dist.all_gather(all_seeds, seeds)
        dist.destroy_process_group()
        q.put((rank, got == own, bool(np.isfinite(blob.numpy()).all()), times,
               len(set(torch.cat(all_seeds).tolist()))))
    except Exception as e:  # surface the failure to the parent
        q.put((rank, repr(e)))


@pytest.mark.timeout(600)
def test_replicas_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=540) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert len(r) == 5, f"rank {r[0]} failed: {r[1]}"
        rank, same, finite, times, n_seeds = r
        assert same and finite, f"rank {rank}: broadcast blob differs from the packed weights"
        assert times == [2.0, 10.0]  # elementwise max over ranks
        assert n_seeds == 64  # utterance noise streams never collide across ranks


@pytest.mark.parametrize("gpus", [2, 8])
def test_bench_gpus_flag_launches_replica_ranks(gpus):
    """`bench.py --gpus 2` outside a torch.distributed environment re-launches itself as 2 ranks
    under torch.distributed.run (a child process, never exec), each rank runs its replica, rank 0
    reports the whole job: n_gpus 2, "replicas x2", global batch 2 x 32, 125-frame utterances and
    at least MIN_JOBS (16) timed jobs whatever --steps asks, with the per-job median / min / max. CPU only: --launcher-selftest swaps in a stand-in engine and gloo."""
    import json
    import subprocess
    import sys

    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", str(gpus), "--launcher-selftest", "--steps",
                        "20", "--warmup", "1"], capture_output=True, text=True, timeout=400,
                       env=dict(os.environ, OMP_NUM_THREADS="1"))
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1  # only rank 0 prints
    out = json.loads(lines[0])
    assert out["n_gpus"] == gpus and out["config"]["parallelism"] == f"replicas x{gpus}"
    assert out["config"]["global_batch"] == 32 * gpus and out["config"]["utterance_frames"] == 125
    assert out["steps"] == 16 * 125 and out["steps_requested"] == 20 and out["scaling"] == "weak"
    pj = out["per_job"]
    assert pj["jobs"] == 16 and pj["min"] <= pj["median"] <= pj["max"]
