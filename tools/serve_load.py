#!/usr/bin/env python3
"""HTTP load test of the serving front end on ONE GPU (BASELINE configs[3] at one GPU's share:
256 utterances over 8 GPUs = 32 concurrent streams per GPU; the 8-GPU node is the driver's).

The launcher never touches the GPU. It starts (1) the server, `python -m pocket_tts_amd.serve`
(real engine, pipelined, 32 slots, a synthetic 125-frame voice prompt) on 127.0.0.1, and (2)
client processes, so the load generator does not share the server's interpreter. Each client
thread POSTs /stream (chunked 16-bit PCM) with 40 token ids and eos_threshold = +1e9 (no EOS:
each request runs its max_gen_len = 22 * 13 = 286 frames, the tts_model.rs:968-969 rule for the 20
words stated with the ids), CLOSED LOOP: each of the 32 streams issues its next request as soon as
the previous one ends, for --seconds per round, so a round is a steady state of continuous
batching (slots recycled as requests finish and new ones are admitted in small groups) rather than
one synchronized burst. Reports per round the audio-sec/wall-sec through HTTP (audio of the
requests that completed inside the round / round wall time) and the p50 / p90 time to first chunk
(burst: the first request of each stream, all released together; steady: every later request),
and the median over rounds.

  python tools/serve_load.py [--clients 32] [--procs 4] [--rounds 3] [--seconds 6] [--port 8765] [--out f.json]"""

import argparse
import json
import os
import subprocess
import sys
import threading
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(HERE, "..", "pocket-tts_amd")


def ids(i):
    return [(k * 97 + 13 + 7 * i) % 4000 for k in range(40)]


def client(port, first, n, t_go, seconds):
    """n streams (ids first..first+n-1) in threads, all released at wall time t_go (shared by
    every client process), each issuing requests back to back until t_go + seconds; prints one
    JSON line: per stream, the list of its requests."""
    import httpx

    base = f"http://127.0.0.1:{port}"
    out = [None] * n
    # one client per thread, built and connected before the clock starts (building an httpx
    # client loads a CA bundle: ~tens of ms under the GIL, which is client cost, not serving)
    clients = [httpx.Client(timeout=300.0) for _ in range(n)]
    for c in clients:
        c.get(base + "/health")
    go = threading.Barrier(n)

    def one(j):
        go.wait()
        time.sleep(max(0.0, t_go - time.time()))
        reqs = []
        while time.time() < t_go + seconds:
            t0 = time.time()
            t_first, nbytes = None, 0
            body = {"token_ids": ids(first + j + 97 * len(reqs)), "words": 20, "eos_threshold": 1e9}
            with clients[j].stream("POST", base + "/stream", json=body) as r:
                r.raise_for_status()
                t_hdr = time.time()
                t_route = float(r.headers.get("X-PTTS-Route-Time", "nan"))
                for chunk in r.iter_bytes():
                    if t_first is None and chunk:
                        t_first = time.time()
                    nbytes += len(chunk)
            reqs.append({"start": t0, "first": t_first, "end": time.time(), "samples": nbytes // 2,
                         "route": t_route, "headers": t_hdr})
        out[j] = reqs

    ts = [threading.Thread(target=one, args=(j,)) for j in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=32)
    ap.add_argument("--procs", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--seconds", type=float, default=6.0, help="closed-loop duration of one round")
    ap.add_argument("--port", type=int, default=8765)
    ap.add_argument("--out", default="")
    ap.add_argument("--workdir", default=os.path.join(HERE, "..", "gpurun_out"))
    ap.add_argument("--back-frames", type=int, default=2, help="the server's frames per Mimi decode pass")
    ap.add_argument("--preview-rows", type=int, default=8, help="the server's first-frame preview rows (0: off)")
    ap.add_argument("--trace", action="store_true",
                    help="run the server with PTTS_SERVE_TRACE=1 and report the medians of its per-request "
                         "submit -> admission and submit -> first frame times")
    args = ap.parse_args()

    import httpx

    os.makedirs(args.workdir, exist_ok=True)
    prompt_path = os.path.join(args.workdir, "serve_load_prompt.npy")
    np.save(prompt_path, (0.11 * np.random.default_rng(1).standard_normal((125, 1024))).astype(np.float32))
    env = dict(os.environ, PYTHONPATH=os.path.abspath(PKG) + os.pathsep + os.environ.get("PYTHONPATH", ""))
    if args.trace:
        env["PTTS_SERVE_TRACE"] = "1"
    log_path = os.path.join(args.workdir, "serve_load_server.log")
    log = open(log_path, "w")
    server = subprocess.Popen([sys.executable, "-m", "pocket_tts_amd.serve", "--voice", f"synth={prompt_path}",
                               "--slots", "32", "--max-ctx", "480", "--port", str(args.port),
                               "--back-frames", str(args.back_frames), "--preview-rows", str(args.preview_rows)],
                              env=env, stdout=log, stderr=subprocess.STDOUT)
    try:
        base = f"http://127.0.0.1:{args.port}"
        for _ in range(1200):  # first import torch / engine build on a fresh box can take a while
            if server.poll() is not None:
                raise SystemExit(f"server exited with {server.returncode}")
            try:
                if httpx.get(base + "/health", timeout=1.0).status_code == 200:
                    break
            except httpx.HTTPError:
                time.sleep(0.1)
        result = {"clients": args.clients, "procs": args.procs, "route": "/stream", "seconds_per_round": args.seconds,
                  "back_frames": args.back_frames, "preview_rows": args.preview_rows, "rounds": []}
        per = [args.clients // args.procs + (1 if p < args.clients % args.procs else 0) for p in range(args.procs)]
        for rnd in range(args.rounds):
            procs, first = [], 0
            t_go = time.time() + 3.0  # client processes start, import httpx and connect first
            h0 = httpx.get(base + "/health", timeout=5.0).json()
            for n in per:
                procs.append(subprocess.Popen([sys.executable, __file__, "client", str(args.port), str(first), str(n),
                                               repr(t_go), repr(args.seconds)], stdout=subprocess.PIPE, text=True))
                first += n
            streams = []
            h1 = None
            for p in procs:
                o, _ = p.communicate(timeout=600)
                if p.returncode != 0:
                    raise SystemExit(f"client failed ({p.returncode})")
                streams += json.loads(o.strip().splitlines()[-1])
            h1 = httpx.get(base + "/health", timeout=5.0).json()
            reqs = [q for st in streams for q in st]
            t0 = min(q["start"] for q in reqs)
            wall = max(q["end"] for q in reqs) - t0
            samples = sum(q["samples"] for q in reqs)
            burst = sorted(st[0]["first"] - st[0]["start"] for st in streams)
            steady = sorted(q["first"] - q["start"] for st in streams for q in st[1:])
            pct = lambda v, f: round(1e3 * v[min(len(v) - 1, int(f * (len(v) - 1)))], 2) if v else None
            rec = {"round": rnd, "wall_s": round(wall, 3), "requests": len(reqs), "audio_s": round(samples / 24000.0, 2),
                   "audio_sec_per_wall_sec": round(samples / 24000.0 / wall, 2),
                   "frames_per_request": reqs[0]["samples"] // 1920,
                   "ttfc_burst_p50_ms": pct(burst, 0.5), "ttfc_burst_p90_ms": pct(burst, 0.9),
                   "ttfc_steady_p50_ms": pct(steady, 0.5), "ttfc_steady_p90_ms": pct(steady, 0.9)}
            lat = [(q["route"] - q["start"], q["headers"] - q["start"], q["first"] - q["route"]) for st in streams
                   for q in st[1:] if q["route"] == q["route"]]
            if lat:  # where a steady request's time to first chunk goes (client and server share a clock)
                med3 = np.median(np.array(lat), axis=0)
                rec.update({"steady_start_to_route_ms": round(1e3 * med3[0], 2),
                            "steady_start_to_headers_ms": round(1e3 * med3[1], 2),
                            "steady_route_to_first_chunk_ms": round(1e3 * med3[2], 2)})
            if "steps" in h0:  # the scheduler's own counters over the round (3-s start-up included)
                ds, df = h1["steps"] - h0["steps"], h1["frames"] - h0["frames"]
                rec.update({"server_steps": ds, "server_rows_per_step": round(df / max(ds, 1), 2),
                            "server_ms_per_step": round(1e3 * (wall) / max(ds, 1), 4)})
            result["rounds"].append(rec)
            print(json.dumps(rec), flush=True)
        med = lambda k: float(np.median([r[k] for r in result["rounds"] if r[k] is not None]))
        result["median"] = {k: round(med(k), 2) for k in ("audio_sec_per_wall_sec", "ttfc_burst_p50_ms",
                                                          "ttfc_steady_p50_ms", "ttfc_steady_p90_ms")}
        if args.trace:  # the server's own per-request stamps (serve.py BatchScheduler._deliver)
            log.flush()
            tr = {"admit_wait_ms": [], "start_ms": [], "first_after_start_ms": [], "first_ms": [], "first_to_chunk0_ms": []}
            for line in open(log_path):
                if line.startswith("ptts-serve slot"):
                    w = line.split()
                    for k in tr:
                        if k in w:
                            tr[k].append(float(w[w.index(k) + 1]))
            result["server_trace_median"] = {k: round(float(np.median(v)), 3) for k, v in tr.items() if v}
            result["server_trace_median"]["requests"] = len(tr["first_ms"])
        print(json.dumps({"median": result["median"], "trace": result.get("server_trace_median")}), flush=True)
        r = httpx.post(base + "/v1/audio/speech", json={"token_ids": ids(0), "words": 20, "response_format": "wav"}, timeout=120)
        r.raise_for_status()
        result["openai_wav_bytes"] = len(r.content)
        if args.out:
            json.dump(result, open(args.out, "w"), indent=1)
    finally:
        server.terminate()
        try:
            server.wait(timeout=30)
        except subprocess.TimeoutExpired:
            server.kill()


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "client":
        client(int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), float(sys.argv[5]), float(sys.argv[6]))
    else:
        main()
