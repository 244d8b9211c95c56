#!/usr/bin/env python3
"""TEST INFRASTRUCTURE ONLY: the CPU baseline leg of bench.py (fallback 3).

The reference's Candle CPU path cannot be built here (no cargo, no crates), so the baseline is the
repo's C restatement of the reference algorithm (oracle/libptts_oracle.so, fp32, kind "port"), run
on the configs[2] job exactly as the GPU bench runs it, per utterance:

  voice state precomputed (the 125-frame prompt prefill is untimed, as on the GPU where the voice
  KV is copied in), then TIMED: 40-token text prefill + 125 generated frames (forced, no EOS),
  temp 0.7 noise replaced by the deterministic temp-0 path (the per-frame cost is the same).

Two builds of the same C source (oracle/Makefile):
  blocked   libptts_cpu_fast.so (-DORC_FAST): cache-blocked AVX2/FMA GEMMs for every linear and
            conv (the form candle's gemm crate gives the reference on a CPU). The headline value.
  plain     libptts_oracle.so, the checker: unblocked dot loops, no FMA contraction. Reported
            beside it (a bounded 40-frame sample).
Two layouts:
  per-core  P single-thread worker processes (OMP_NUM_THREADS=1), each pinned to its own core, U
            utterances each in sequence, started together; value = P x U x 10 s / (last end -
            first start). P is the box's CPU share (16 on a 1-GPU box: the harness sizes worker
            pools to it), U = 2, so the 32 utterances of the GPU's B = 32 job run on 16 cores.
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


def _oracle(lib_name):
    sys.path.insert(0, str(ROOT / "tests"))
    from _oracle import Oracle

    return Oracle(0x5EED, lib_name=lib_name)


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


def worker(core, u0, n_utt, frames, lib_name):
    """One pinned single-thread process: setup (untimed voice prefill of its utterances), report
    ready, wait for go, run its utterances one after another, report times."""
    if core >= 0:
        os.sched_setaffinity(0, {core})
    o = _oracle(lib_name)
    states = []
    for u in range(u0, u0 + n_utt):
        prompt, ids = _job_inputs(u)
        s = o.new_state(PROMPT_FRAMES + TEXT_TOKENS + frames + 8)
        s.prefill(prompt)
        states.append((s, ids))
    print("ready", flush=True)
    sys.stdin.readline()
    t0 = time.monotonic()
    for s, ids in states:
        s.prefill_tokens(ids)
        lat = None
        for _ in range(frames):
            lat = s.step(lat)["latent"]
    print(json.dumps({"t0": t0, "t1": time.monotonic()}), flush=True)


def per_core(procs, frames, utts_per_proc=1, lib_name="libptts_oracle.so"):
    cores = sorted(os.sched_getaffinity(0))[:procs]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    ps = [subprocess.Popen([sys.executable, __file__, "--worker", str(c), str(i * utts_per_proc), str(utts_per_proc),
                            str(frames), lib_name], env=env, stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
          for i, c in enumerate(cores)]
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


def all_core(n_utt, threads, frames, lib_name):
    os.environ["OMP_NUM_THREADS"] = str(threads)
    o = _oracle(lib_name)
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
    ap.add_argument("--utts-per-proc", type=int, default=2, help="per-core layout: utterances per process")
    ap.add_argument("--allcore-utts", type=int, default=2, help="all-core layout: utterances in sequence")
    ap.add_argument("--frames", type=int, default=125)
    ap.add_argument("--plain-frames", type=int, default=40, help="bounded sample of the unblocked checker build")
    ap.add_argument("--scaling-procs", default="1,4",
                    help="per-core layout at these process counts too (1 utterance each): the per-core rate's "
                         "scaling over the share, which the 32-process and whole-host figures extrapolate")
    ap.add_argument("--worker", nargs=5, help=argparse.SUPPRESS)
    a = ap.parse_args()
    if a.worker:
        c, u0, n, f, lib_name = a.worker
        worker(int(c), int(u0), int(n), int(f), lib_name)
        return
    share = len(os.sched_getaffinity(0))
    procs = max(1, min(a.procs, share))
    fast, plain = "libptts_cpu_fast.so", "libptts_oracle.so"
    n, wall = per_core(procs, a.frames, a.utts_per_proc, fast)
    utts = n * a.utts_per_proc
    out = {"value": round(utts * a.frames * 0.08 / wall, 3), "unit": "audio-sec/wall-sec", "cores": n, "kind": "port",
           "build": "blocked (libptts_cpu_fast.so: cache-blocked AVX2/FMA GEMMs, the stand-in for candle's gemm crate)",
           "layout": f"{n} single-thread processes pinned one per core, {a.utts_per_proc} utterances each in sequence "
                     f"({utts} utterances = the GPU job's batch)",
           "sample": f"{utts} utterances x ({TEXT_TOKENS}-token text prefill + {a.frames} frames), voice "
                     f"({PROMPT_FRAMES}-frame prompt) precomputed; fp32 C restatement of the reference "
                     f"(Candle unbuildable offline)",
           "wall_s": round(wall, 3), "per_core_realtime": round(a.frames * 0.08 * a.utts_per_proc / wall, 3),
           "nproc": os.cpu_count(), "affinity_cpus": share, **(physical_cores() or {})}
    if a.plain_frames > 0:
        n2, w2 = per_core(procs, a.plain_frames, 1, plain)
        out["plain_build"] = {"value": round(n2 * a.plain_frames * 0.08 / w2, 3), "unit": "audio-sec/wall-sec",
                              "cores": n2, "wall_s": round(w2, 3),
                              "build": "libptts_oracle.so (the checker: unblocked dot loops, no FMA contraction)",
                              "sample": f"{n2} utterances x ({TEXT_TOKENS}-token prefill + {a.plain_frames} frames), "
                                        f"one per pinned single-thread process"}
    # BASELINE.md §4.2 also names 32 pinned single-thread processes (one per utterance of B = 32)
    # and a whole-host run; the harness caps a 1-GPU box's worker pools at its 16-core share, so
    # those are not run: the per-core rate is measured at fewer processes as well, and the larger
    # layouts are stated as that rate x cores (labelled extrapolated, never measured)
    scal = {}
    for p_ in [int(v) for v in a.scaling_procs.split(",") if v.strip()]:
        if 1 <= p_ < procs:
            n3, w3 = per_core(p_, a.frames, 1, fast)
            scal[str(n3)] = round(a.frames * 0.08 / w3, 3)  # audio-sec per wall-sec per core
    scal[str(n)] = out["per_core_realtime"]
    out["per_core_scaling"] = {"realtime_per_core_by_procs": scal,
                               "note": "one utterance per pinned single-thread process (the share's own "
                                       "layout: 2 utterances each)"}
    rate = min(scal.values())
    out["extrapolated"] = {
        "per_core_32": {"value": round(32 * rate, 3), "cores": 32,
                        "basis": "32 pinned single-thread processes x the lowest measured per-core rate"},
        "whole_host": {"value": round(rate * (out.get("sockets") or 1) * (out.get("physical_cores_per_socket") or n), 3),
                       "cores": (out.get("sockets") or 1) * (out.get("physical_cores_per_socket") or n),
                       "basis": "every physical core of the host x the lowest measured per-core rate"},
        "measured": False}
    if a.allcore_utts > 0:
        threads = procs
        w = all_core(a.allcore_utts, threads, a.frames, fast)
        out["all_core"] = {"value": round(a.allcore_utts * a.frames * 0.08 / w, 3), "unit": "audio-sec/wall-sec",
                           "threads": threads, "wall_s": round(w, 3), "build": "blocked",
                           "sample": f"{a.allcore_utts} utterances in sequence, OpenMP intra-op threads"}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
