#!/usr/bin/env python3
"""TEST INFRASTRUCTURE ONLY: the CPU baseline leg of bench.py (fallback 3).

The reference's Candle CPU path cannot be built here (no cargo, no crates), so the baseline is the
repo's C restatement of the reference algorithm (oracle/libptts_oracle.so, fp32, kind "port"), run
on the configs[2] job exactly as the GPU bench runs it, per utterance:

  voice state precomputed (the 125-frame prompt prefill is untimed, as on the GPU where the voice
  KV is copied in), then TIMED: 40-token text prefill + 125 generated frames (forced, no EOS),
  temp 0.7 noise replaced by the deterministic temp-0 path (the per-frame cost is the same).

Two layouts:
  per-core  P single-thread worker processes (OMP_NUM_THREADS=1), each pinned to its own core,
            one utterance each, started together; value = P x 10 s / (last end - first start).
  all-core  one process whose OpenMP intra-op threads use every core of the share, utterances one
            after another (Candle's B = 1 intra-op mode); value = n x 10 s / wall.

Run by bench.py as a CHILD process (it never touches the GPU); prints one JSON line.
Usage: python oracle/cpu_baseline.py [--procs P] [--allcore-utts N] [--frames 125]
"""

from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PROMPT_FRAMES, TEXT_TOKENS = 125, 40


def _job_inputs(u):
    import numpy as np

    prompt = (0.11 * np.random.default_rng(1).standard_normal((PROMPT_FRAMES, 1024))).astype(np.float32)
    ids = np.array([(i * 97 + 13 + 7 * u) % 4000 for i in range(TEXT_TOKENS)], np.int32)
    return prompt, ids


def _run_utterance(o, u, frames):
    """Untimed voice prefill, then the timed text prefill + frames; returns (start, end)."""
    prompt, ids = _job_inputs(u)
    s = o.new_state(PROMPT_FRAMES + TEXT_TOKENS + frames + 8)
    s.prefill(prompt)
    t0 = time.monotonic()
    s.prefill_tokens(ids)
    lat = None
    for _ in range(frames):
        lat = s.step(lat)["latent"]
    return t0, time.monotonic()


def worker(core, u, frames):
    """One pinned single-thread process: setup, report ready, wait for go, run, report times."""
    if core >= 0:
        os.sched_setaffinity(0, {core})
    sys.path.insert(0, str(ROOT / "tests"))
    from _oracle import Oracle

    o = Oracle(0x5EED)
    prompt, ids = _job_inputs(u)
    s = o.new_state(PROMPT_FRAMES + TEXT_TOKENS + frames + 8)
    s.prefill(prompt)
    print("ready", flush=True)
    sys.stdin.readline()
    t0 = time.monotonic()
    s.prefill_tokens(ids)
    lat = None
    for _ in range(frames):
        lat = s.step(lat)["latent"]
    print(json.dumps({"t0": t0, "t1": time.monotonic()}), flush=True)


def per_core(procs, frames):
    cores = sorted(os.sched_getaffinity(0))[:procs]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    ps = [subprocess.Popen([sys.executable, __file__, "--worker", str(c), str(i), str(frames)], env=env,
                           stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True) for i, c in enumerate(cores)]
    try:
        for p in ps:
            assert p.stdout.readline().strip() == "ready"
        for p in ps:  # all workers are set up: start them together
            p.stdin.write("go\n")
            p.stdin.flush()
        res = [json.loads(p.stdout.readline()) for p in ps]
    finally:
        for p in ps:
            p.wait(timeout=600)
    wall = max(r["t1"] for r in res) - min(r["t0"] for r in res)
    return len(cores), wall


def all_core(n_utt, threads, frames):
    os.environ["OMP_NUM_THREADS"] = str(threads)
    sys.path.insert(0, str(ROOT / "tests"))
    from _oracle import Oracle

    o = Oracle(0x5EED)
    wall = 0.0
    for u in range(n_utt):
        t0, t1 = _run_utterance(o, u, frames)
        wall += t1 - t0
    return wall


def physical_cores():
    """(sockets, physical cores per socket) from /proc/cpuinfo, None if unreadable."""
    try:
        txt = Path("/proc/cpuinfo").read_text()
    except OSError:
        return None
    phys, cores = set(), None
    for line in txt.splitlines():
        if line.startswith("physical id"):
            phys.add(line.split(":")[1].strip())
        elif line.startswith("cpu cores") and cores is None:
            cores = int(line.split(":")[1])
    return {"sockets": len(phys) or None, "physical_cores_per_socket": cores}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=16, help="per-core layout: worker processes (<= CPU share)")
    ap.add_argument("--allcore-utts", type=int, default=2, help="all-core layout: utterances in sequence")
    ap.add_argument("--frames", type=int, default=125)
    ap.add_argument("--worker", nargs=3, type=int, help=argparse.SUPPRESS)
    a = ap.parse_args()
    if a.worker:
        worker(*a.worker)
        return
    share = len(os.sched_getaffinity(0))
    procs = max(1, min(a.procs, share))
    audio = a.frames * 0.08
    n, wall = per_core(procs, a.frames)
    out = {"value": round(n * audio / wall, 3), "unit": "audio-sec/wall-sec", "cores": n, "kind": "port",
           "layout": f"{n} single-thread processes pinned one per core, one utterance each",
           "sample": f"{n} utterances x ({TEXT_TOKENS}-token text prefill + {a.frames} frames), voice "
                     f"({PROMPT_FRAMES}-frame prompt) precomputed; fp32 C restatement of the reference "
                     f"(Candle unbuildable offline)",
           "wall_s": round(wall, 3), "nproc": os.cpu_count(), "affinity_cpus": share, **(physical_cores() or {})}
    if a.allcore_utts > 0:
        threads = procs
        w = all_core(a.allcore_utts, threads, a.frames)
        out["all_core"] = {"value": round(a.allcore_utts * audio / w, 3), "unit": "audio-sec/wall-sec",
                           "threads": threads, "wall_s": round(w, 3),
                           "sample": f"{a.allcore_utts} utterances in sequence, OpenMP intra-op threads"}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
