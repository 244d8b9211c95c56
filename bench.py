#!/usr/bin/env python3
"""Throughput bench of the Pocket TTS generation hot path (BASELINE.json configs[2]).

Workload per GPU: 32 concurrent utterances (batch rows), each a synthetic "10 s" utterance:
voice prompt [125 x 1024] ~ N(0, 0.11^2), 40 text tokens, generation forced to 125 frames
(eos_threshold = +inf), temperature 0.7, lsd_decode_steps 1, synthetic weights (seed 0x5EED;
real checkpoints are gated/offline). One "step" = one batched iteration of the
generate_stream_segment loop body (tts_model.rs:1006-1070) for all 32 rows: FlowLM step +
flow head + Mimi decode -> 32 x 1920 PCM samples (32 x 80 ms of audio), copied to pinned host
memory inside the step (the graphs end in async D2H copies; fetch() reads host memory).

The utterance length is fixed at 125 frames whatever --steps says: a timed job is the admission of
all B utterances (voice-KV copy + 40-token text prefill per row) followed by the 125 batched steps
that deliver their 10 s of audio. --steps K times max(MIN_JOBS, ceil(K / 125)) such jobs back to
back (MIN_JOBS = 16, >= 1 s of GPU work, so one scheduling hiccup cannot move the line by
percent); `steps` in the output is the number of steps actually timed (`steps_requested` = K).
value = audio seconds produced by all ranks / max-over-ranks wall time of all timed jobs;
`per_job` gives the median, min and max of the per-job values (each job's time max over ranks).
The voice state is precomputed (as in configs[1]); warmup = one short job of W steps on the same
rows.

Any PTTS_* environment variable, or a library whose build id differs from the checked-out
sources (a stale binary or a -DPTTS_PROBES measurement build), marks the line "NOT A PRODUCT RUN"
and lists them under `tuned`.

Multi-GPU (--gpus N): replicas (independent utterances per GPU, no per-step collective). Without
a torch.distributed environment the process re-launches itself as N ranks under
`torch.distributed.run` (a child process; this parent never touches the GPU); rank 0 builds the
weights and broadcasts the packed blob over RCCL once at load time.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

# the HIP runtime reads this at its initialization, which torch.distributed's RCCL setup (N > 1)
# does before the engine library is loaded (the library sets the same default at load: capi.cpp)
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "pocket-tts_amd"))
sys.path.insert(0, str(ROOT / "tests"))

METRIC = "audio-sec/wall-sec (RTF) per GPU at batch=32 + p50 first-chunk latency"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8 TB/s spec
F32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: fp32 matrix/vector peak
BATCH, PROMPT_FRAMES, TEXT_TOKENS, UTT_FRAMES = 32, 125, 40, 125  # 125 frames = 10 s per utterance
MIN_JOBS = 16  # timed jobs per run whatever --steps says (~1.3 s of GPU work at B = 32)


def measured_traffic(op):
    """HBM bytes per launch of `op` from the committed rocprofv3 PMC passes (FETCH_SIZE x 2 +
    WRITE_SIZE, MI355X_MICROARCH.md HBM section), produced by tools/prof_ops.py; None if the op
    was not profiled."""
    path = ROOT / "profiles" / "traffic.json"
    if not path.exists():
        return None, None
    t = json.load(open(path))
    if op not in t.get("ops", {}):
        return None, None
    return t["ops"][op]["hbm_bytes_per_launch"], t.get("source")


def measured_in_step(op):
    """Average duration (us) of `op`'s launches inside the pipelined step, where it shares the CUs
    with the other part, from the committed rocprofv3 --kernel-trace of the bench
    (profiles/op_stats.csv, tools/prof_ops.py piped); None if absent."""
    path = ROOT / "profiles" / "op_stats.csv"
    if not path.exists():
        return None
    import csv
    for r in csv.DictReader(open(path)):
        if r["op"] == op:
            return float(r["rocprof_avg_us"])
    return None


def measured_in_step_all():
    """{op: average in-step duration (us)} from the committed kernel trace (profiles/op_stats.csv)."""
    path = ROOT / "profiles" / "op_stats.csv"
    if not path.exists():
        return {}
    import csv
    return {r["op"]: float(r["rocprof_avg_us"]) for r in csv.DictReader(open(path)) if r["rocprof_avg_us"]}


def kernel_aggregates(top=3):
    """Per kernel (template instance) over the committed in-step trace (profiles/op_stats.csv): its
    total time per step pass (sum over its ops of in-step average x launches) and its algorithmic
    flops / bytes over the same launches, ranked by total time. The first entry is the kernel that
    dominates the GPU time of the measured step; its fraction is its total work over its total
    time against the peak of its bound (MFMA for flop-heavy kernels, HBM otherwise)."""
    path = ROOT / "profiles" / "op_stats.csv"
    if not path.exists():
        return None
    import csv
    agg = {}
    for r in csv.DictReader(open(path)):
        if not r["rocprof_avg_us"]:
            continue
        a = agg.setdefault(r["kernel"], {"us": 0.0, "flops": 0.0, "bytes": 0.0, "launches": 0, "ops": []})
        n = int(r["calls"])
        a["us"] += float(r["rocprof_avg_us"]) * n
        a["flops"] += float(r["flops"] or 0) * n
        a["bytes"] += float(r["bytes"] or 0) * n
        a["launches"] += n
        a["ops"].append(r["op"])
    total = sum(a["us"] for a in agg.values())
    ridge = F32_PEAK_TFLOPS * 1e12 / (HBM_PEAK_GBS * 1e9)
    out = []
    for k, a in sorted(agg.items(), key=lambda kv: -kv[1]["us"])[:top]:
        mfma = a["bytes"] == 0 or a["flops"] / a["bytes"] >= ridge
        ach = a["flops"] / (a["us"] * 1e-6) / 1e12 if mfma else a["bytes"] / (a["us"] * 1e-6) / 1e9
        peak = F32_PEAK_TFLOPS if mfma else HBM_PEAK_GBS
        out.append({"kernel": k, "share_of_gpu_time": round(a["us"] / total, 4), "launches": a["launches"],
                    "avg_us": round(a["us"] / a["launches"], 2), "bound": "mfma" if mfma else "hbm",
                    "achieved": round(ach, 2), "unit": "TFLOP/s" if mfma else "GB/s", "peak": peak,
                    "frac": round(ach / peak, 4), "ops": sorted(set(a["ops"]))})
    return out


def front_bytes(B, K, distinct_voices=1):
    """Algorithmic HBM bytes of one front part (FlowLM step): the f32 step weights once
    (84,527,137 floats) plus the KV the six layers read (49,152 B per cached position = 6 layers x
    8,192 B) at the job's mean context L = prompt + text + K/2, with every distinct voice's
    PROMPT_FRAMES-position prefix counted ONCE (the rows of one voice read its shared cache,
    KvStore::pre) and each row's own text / frame positions per row, plus the 49,152-B append
    per row."""
    L = PROMPT_FRAMES + TEXT_TOKENS + K / 2.0
    return 84_527_137 * 4 + 49_152 * (B * (L - PROMPT_FRAMES) + distinct_voices * PROMPT_FRAMES) + B * 49_152


def step_roofline(plan, B, K, back_frames, steady_us):
    """The roofline of the timed step (per frame): the front part's algorithmic bytes at the HBM peak
    plus the back part's algorithmic flops at the fp32 MFMA peak (serial sum; the two parts overlap
    in the pipelined step, so `overlap_floor_us`, the larger of the two, is the tighter floor), over
    the measured steady step. The front / back in-step fractions divide the same bytes / flops by
    the summed in-step durations of the part's launches (committed kernel trace of this bench)."""
    f_bytes = front_bytes(B, K)
    b_flops = B * (525.1e6 + 65_536 * 266)  # per frame
    f_us = f_bytes / (HBM_PEAK_GBS * 1e9) * 1e6
    b_us = b_flops / (F32_PEAK_TFLOPS * 1e12) * 1e6
    out = {"floor_us": round(f_us + b_us, 1), "front_floor_us": round(f_us, 1), "back_floor_us": round(b_us, 1),
           "overlap_floor_us": round(max(f_us, b_us), 1), "measured_us": round(steady_us, 1),
           "frac": round((f_us + b_us) / steady_us, 4), "frac_overlap": round(max(f_us, b_us) / steady_us, 4)}
    ins = measured_in_step_all()
    names = [n for n, _, _ in plan]
    front = [n for n in names if n.startswith(("flow.", "head.", "front_commit"))]
    back = [n for n in names if n.startswith(("mimi.", "seanet.")) or n == "commit"]
    if ins and all(n in ins for n in front + back):
        fu = sum(ins[n] for n in front)
        bu = sum(ins[n] for n in back) / back_frames  # a back pass decodes back_frames frames
        out["front_in_step"] = {"sum_launch_us": round(fu, 1), "achieved": round(f_bytes / (fu * 1e-6) / 1e9, 1),
                                "unit": "GB/s", "frac": round(f_bytes / (fu * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)}
        out["back_in_step"] = {"sum_launch_us_per_frame": round(bu, 1),
                               "achieved": round(b_flops / (bu * 1e-6) / 1e12, 2), "unit": "TFLOP/s",
                               "frac": round(b_flops / (bu * 1e-6) / 1e12 / F32_PEAK_TFLOPS, 4)}
        out["source"] = "profiles/op_stats.csv (rocprofv3 --kernel-trace of bench.py, tools/prof_ops.py piped)"
    return out


def measured_mfma():
    """Per-op MFMA busy cycles from the committed rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES pass
    (tools/prof_ops.py mfma), {} if absent."""
    path = ROOT / "profiles" / "mfma.json"
    return json.load(open(path))["ops"] if path.exists() else {}


def phase_rooflines(per_op, plan, B, K, back_frames=1):
    """SURVEY §8(d) per-phase rooflines over one batched step, from the per-op HIP-event times
    (each op timed alone; the plan lists every launch of the step, repeated ops counted per launch):
    - front (FlowLM step + flow head): HBM-bound; algorithmic bytes = front_bytes(): the FlowLM
      per-step weights (84,527,137 f32) + the KV read at the job's mean context, the shared voice
      prefix once, and the per-row append;
    - back (Mimi decode): MFMA-bound; algorithmic flops = 525.1 MFLOP per frame (GEMMs and convs)
      + 65,536 per window key (W = 266) of window attention, per row and frame; a back pass covers
      back_frames frames."""
    us = {n: u for u, n, _, _ in per_op}
    front = sum(us[n] for n, _, _ in plan if n.startswith(("flow.", "head.", "front_commit")))
    back = sum(us[n] for n, _, _ in plan if n.startswith(("mimi.", "seanet.")) or n == "commit")
    f_bytes = front_bytes(B, K)
    b_flops = back_frames * B * (525.1e6 + 65_536 * 266)
    fa = f_bytes / (front * 1e-6) / 1e9
    ba = b_flops / (back * 1e-6) / 1e12
    mf = measured_mfma()  # rocprof MFMA busy over the back ops, against 1,024 SIMDs at 2.4 GHz
    bops = [n for n, _, _ in plan if (n.startswith(("mimi.", "seanet.")) or n == "commit") and n in mf]
    busy = sum(mf[n]["mfma_busy_cycles"] for n in bops)
    dur = sum(mf[n]["rocprof_avg_us"] for n in bops)
    return {
        "front": {"bound": "hbm", "algorithmic_bytes": round(f_bytes), "sum_op_us": round(front, 1),
                  "achieved": round(fa, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(fa / HBM_PEAK_GBS, 4)},
        "back": {"bound": "mfma", "algorithmic_flops": round(b_flops), "sum_op_us": round(back, 1),
                 "achieved": round(ba, 2), "peak": F32_PEAK_TFLOPS, "unit": "TFLOP/s",
                 "frac": round(ba / F32_PEAK_TFLOPS, 4),
                 "rocprof_mfma_busy_frac": round(busy / (1024 * 2.4e9 * dur * 1e-6), 4) if dur else None},
    }


def slot_seed(round_id, rank, row):
    """Noise-stream seed of one utterance: distinct across jobs, ranks and rows."""
    return 100000 * round_id + 1000 * rank + row + 1


def broadcast_weights(dist, blob):
    """The one collective of the replicas design: rank 0's packed weight blob to every rank
    (RCCL over xGMI on GPUs; gloo in the CPU tests)."""
    dist.broadcast(blob, src=0)


def max_over_ranks(dist, values, device):
    """Max over ranks of per-rank wall times (the slowest replica bounds the job)."""
    import torch

    t = torch.tensor(values, dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(v) for v in t.tolist()]


def synth_prompt(n=PROMPT_FRAMES, seed=1):
    return (0.11 * np.random.default_rng(seed).standard_normal((n, 1024))).astype(np.float32)


def text_ids(slot):
    return np.array([(i * 97 + 13 + 7 * slot) % 4000 for i in range(TEXT_TOKENS)], np.int32)


class _SelftestEngine:
    """--launcher-selftest only: a CPU stand-in with the Engine surface bench.py drives, so the
    multi-rank launch, the gloo collectives and the output line can be checked without a GPU. It
    computes nothing and the line it yields says so (data: "launcher selftest")."""

    def __init__(self, max_slots, **_):
        self.n = max_slots

    @staticmethod
    def weight_blob_bytes():
        return 4096

    def finalize(self):
        pass

    def voice_from_prompt(self, prompt):
        return object()

    def open_many(self, slots, voices, ids, params):
        self.frames = {s: 0 for s in slots}
        self.max = {s: p.max_frames for s, p in zip(slots, params)}

    def frame_lag(self):
        return 0, 0

    def step_async(self, n):
        time.sleep(2e-4)
        for s in self.frames:
            self.frames[s] += 1
        self.done = np.array([self.frames[s] >= self.max[s] for s in range(n)])  # this call's frame

    def flush_async(self, n):
        time.sleep(1e-4)

    def sync(self):
        pass

    def fetch(self, n):
        import types

        return types.SimpleNamespace(valid=self.done, last=self.done, pcm=np.zeros((n, 1920), np.float32))

    def close(self):
        pass


def free_port():
    import socket

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_replicas(n):
    """--gpus N without a torch.distributed environment: re-run this script as N ranks under
    torch.distributed.run, as a CHILD process (never exec: the driver forbids replacing a process;
    this parent has not touched the GPU), and return its exit code."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={free_port()}", str(Path(__file__).resolve()),
           *sys.argv[1:]]
    return subprocess.run(cmd, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")).returncode


def cpu_baseline_leg(procs):
    """oracle/cpu_baseline.py in a child process (CPU only): like-for-like configs[2] jobs."""
    import subprocess

    r = subprocess.run([sys.executable, str(ROOT / "oracle" / "cpu_baseline.py"), "--procs", str(procs)],
                       capture_output=True, text=True, timeout=900)
    if r.returncode != 0:
        raise RuntimeError("cpu baseline failed: " + r.stderr[-2000:])
    return json.loads(r.stdout.strip().splitlines()[-1])


def _refwav():
    """The reference's assets/ref.wav as held by tests/golden/ref_voice.safetensors (int16, 48 kHz,
    the whole file; gen_golden.py refdata)."""
    from safetensors.numpy import load_file

    g = load_file(str(ROOT / "tests" / "golden" / "ref_voice.safetensors"))
    return g["refwav_i16"].astype(np.float32) / np.float32(32768.0), 48000


def voice_state_bench(pt, dev, reps=5):
    """configs[4]'s voice-cloning leg, as the reference times it (benches/voice_state_bench.rs:4-37:
    get_voice_state_from_tensor on N(0, 1) audio of 3, 15 and 60 s; full_benchmark.rs:22-24:
    get_voice_state(ref.wav)): PCM on the host -> [resample] -> adaptive chunked Mimi encode ->
    speaker projection -> FlowLM prompt prefill -> voice KV in HBM, synchronised, median of `reps`
    after one warm call, on a 1-slot engine with max_ctx 1024 (the reference's default)."""
    e = pt.Engine(device=dev, max_slots=1, max_ctx=1024, lsd_decode_steps=1, seed=0x5EED)
    out = {}
    try:
        cases = [(f"{secs}s_randn", np.random.default_rng(secs).standard_normal(24000 * secs).astype(np.float32),
                  24000) for secs in (3, 15, 60)]
        cases.append(("ref_wav", *_refwav()))
        for name, x, sr in cases:
            e.voice_from_audio(x, sr).close()
            e.sync()
            ts, frames = [], 0
            for _ in range(reps):
                t = time.perf_counter()
                v = e.voice_from_audio(x, sr)
                e.sync()
                ts.append(time.perf_counter() - t)
                frames = v.n_frames
                v.close()
            out[name] = {"median_ms": round(1000 * float(np.median(ts)), 3), "min_ms": round(1000 * min(ts), 3),
                         "audio_s": round(x.size / sr, 3), "sample_rate": sr, "frames": frames}
    finally:
        e.close()
    return out


def text_e2e_bench(pt, dev, reps=3):
    """The reference's generation benchmark (benches/full_benchmark.rs:30-56): TTSModel.generate of a
    short, a medium and a long text on the voice of ref.wav, temp 0, on the SEQUENTIAL engine (one
    utterance, ptts_step per frame: the reference's own loop), host tokenizer + sentence chunking +
    per-chunk prefill + the EOS rule included. Tokenizer: the reference's Unigram/Metaspace
    pipeline (text.py) over the synthetic vocabulary of tests/golden/text_ids.json (the real
    tokenizer.model is not shipped). Two EOS settings: the reference's default threshold -4.0 (with
    synthetic weights the EOS logit exceeds it at once, so a chunk ends after its EOS tail) and no
    EOS (every chunk runs to max_gen_len = (words + 2) * 13, the reference's cap)."""
    from pocket_tts_amd.text import Metaspace, Tokenizer, Unigram

    g = json.load(open(ROOT / "tests" / "golden" / "text_ids.json"))["synthetic"]
    tok = Tokenizer(Unigram([tuple(v) for v in g["vocab"]], g["unk_id"], True), Metaspace())
    e = pt.Engine(device=dev, max_slots=1, max_ctx=1024, lsd_decode_steps=1, seed=0x5EED)
    texts = {"short": "Hello world",
             "medium": "This is a medium length sentence for benchmarking the text to speech system.",
             "long": "The quick brown fox jumps over the lazy dog. " * 10}
    out = {}
    try:
        m = pt.TTSModel(e, temp=0.0, lsd_decode_steps=1, eos_threshold=-4.0, noise_clamp=None, tokenizer=tok)
        voice = m.get_voice_state_from_tensor(*_refwav())
        for eos_name, thr in (("eos_default", -4.0), ("no_eos", float("inf"))):
            m.eos_threshold = thr
            res = {}
            for name, text in texts.items():
                m.generate(text, voice)  # warm (graphs of this row count)
                ts, ttfc, n = [], [], 0
                for _ in range(reps):
                    t = time.perf_counter()
                    first, n = None, 0
                    for fr in m.generate_stream(text, voice):
                        if first is None:
                            first = time.perf_counter() - t
                        n += fr.shape[-1]
                    ts.append(time.perf_counter() - t)
                    ttfc.append(first)
                wall = float(np.median(ts))
                res[name] = {"chars": len(text), "chunks": len(m.split_into_best_sentences(text)),
                             "frames": n // 1920, "audio_s": round(n / 24000.0, 3), "median_ms": round(1000 * wall, 2),
                             "rtf": round(n / 24000.0 / wall, 2),
                             "first_chunk_ms": round(1000 * float(np.median(ttfc)), 3)}
            out[eos_name] = res
    finally:
        e.close()
    return out


def cpu_voice_leg(procs):
    """oracle/cpu_baseline.py --voice in a child process: the CPU port's voice-state time."""
    import subprocess

    r = subprocess.run([sys.executable, str(ROOT / "oracle" / "cpu_baseline.py"), "--voice", "--procs", str(procs)],
                       capture_output=True, text=True, timeout=900)
    if r.returncode != 0:
        raise RuntimeError("cpu voice baseline failed: " + r.stderr[-2000:])
    return json.loads(r.stdout.strip().splitlines()[-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=UTT_FRAMES,
                    help="steps to time: ceil(steps / 125) whole jobs of 125-frame utterances")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=BATCH)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-procs", type=int, default=16, help="CPU baseline worker processes (<= CPU share)")
    ap.add_argument("--no-latency", action="store_true")
    ap.add_argument("--ops-out", default="", help="write per-op timings of the step plan (JSON)")
    ap.add_argument("--no-op-times", action="store_true", help="skip the per-op HIP-event pass (PMC runs)")
    ap.add_argument("--no-quant-variant", action="store_true",
                    help="skip the extra jobs on the int8-weight (weight_quant = QUANT_FLOW_LM), fp8_gemm and "
                         "back_bf16 engines")
    ap.add_argument("--back-frames", type=int, default=4, choices=(1, 2, 4, 8),
                    help="frames per Mimi-decode pass of pipelined stepping (ptts_engine_config.back_frames; "
                         "4, the throughput configuration: 0.505 ms per steady step against 0.522 with 2, 0.529 "
                         "with 8 and 0.62 with 1, DESIGN.md section 14)")
    ap.add_argument("--back-mfma", choices=("f32", "f32x6"), default="f32",
                    help="the back part's f32 GEMMs: f32 MFMA, or f32 products from exact three-piece bf16 "
                         "splits (ptts_engine_config.back_mfma PTTS_BACK_F32X6, f32 accuracy)")
    ap.add_argument("--no-flush", action="store_true",
                    help="drain each job's last frames with step calls (front parts of finished rows run and "
                         "their frames are discarded) instead of ptts_flush_async")
    ap.add_argument("--no-overlap-admission", action="store_true",
                    help="admit each job only after the previous job's last frame is fetched (no overlap of "
                         "its text prefill with that job's last back passes)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="sequential stepping (no FlowLM / Mimi overlap across consecutive frames)")
    ap.add_argument("--profile-frames", type=int, default=0,
                    help="profiling runs only (rocprofv3 PMC passes): utterances of this many frames instead of "
                         "125; the line then says so and is not the configs[2] measurement")
    ap.add_argument("--no-distinct-voices", action="store_true",
                    help="skip the variant job with B distinct voices (one 125-frame prompt per row)")
    ap.add_argument("--no-voice-bench", action="store_true",
                    help="skip the voice-state timing (3/15/60 s randn PCM and ref.wav -> voice KV; configs[4])")
    ap.add_argument("--no-text-bench", action="store_true",
                    help="skip the text-driven generate() timing (short / medium / long, EOS on)")
    ap.add_argument("--launcher-selftest", action="store_true",
                    help="CPU-only check of the N-rank launch path (gloo, stand-in engine; measures nothing)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_replicas(args.gpus))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench: WORLD_SIZE={world} overrides --gpus {args.gpus}", file=sys.stderr)
    selftest = args.launcher_selftest
    dev = "cpu" if selftest else f"cuda:{local_rank}"
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist

        if not selftest:
            torch.cuda.set_device(local_rank)
        dist.init_process_group("gloo" if selftest else "nccl")

    if selftest:
        import types

        pt = types.SimpleNamespace(Engine=_SelftestEngine, GenerationParams=__import__("types").SimpleNamespace)
        args.no_cpu_baseline = args.no_latency = args.no_op_times = args.no_quant_variant = True
        args.no_distinct_voices = args.no_voice_bench = args.no_text_bench = True
    else:
        import pocket_tts_amd as pt

    B, W = args.batch, args.warmup
    K = args.profile_frames if args.profile_frames > 0 else UTT_FRAMES
    jobs = max(MIN_JOBS, -(-args.steps // K)) if args.profile_frames <= 0 else 1
    pipeline = not args.no_pipeline
    back_frames = args.back_frames if pipeline else 1
    back_mfma = {"f32": 0, "f32x6": 2}[args.back_mfma]
    max_ctx = PROMPT_FRAMES + TEXT_TOKENS + K + 8

    def params(round_id, b, n_frames):
        return pt.GenerationParams(temp=0.7, eos_threshold=float("inf"), frames_after_eos=3, max_frames=n_frames,
                                   seed=slot_seed(round_id, rank, b))

    # ---- engine (+ one RCCL broadcast of the packed weights at load time)
    if dist is None:
        eng = pt.Engine(device=local_rank, max_slots=B, max_ctx=max_ctx, lsd_decode_steps=1, seed=0x5EED,
                        pipeline=pipeline, back_frames=back_frames, back_mfma=back_mfma)
    else:
        import torch

        blob = torch.empty(pt.Engine.weight_blob_bytes() // 4, dtype=torch.float32, device=dev)
        eng = pt.Engine(device=local_rank, max_slots=B, max_ctx=max_ctx, lsd_decode_steps=1, seed=0x5EED,
                        weight_blob=blob.data_ptr(), defer_weights=(rank != 0), pipeline=pipeline,
                        back_frames=back_frames, back_mfma=back_mfma)
        if not selftest:
            torch.cuda.synchronize()
        broadcast_weights(dist, blob)
        if not selftest:
            torch.cuda.synchronize()
        if rank != 0:
            eng.finalize()

    def barrier():
        if dist is not None:
            if not selftest:
                import torch

                torch.cuda.synchronize()
            dist.barrier()

    def timed_job(eng, distinct_voices=False):
        """Warmup job, then the timed ones: per job, admission of all B utterances (voice KV prefix +
        text prefill) and the 125 batched steps of their 10 s of audio, i.e. first prefill to last
        PCM frame (in pinned host memory) of B utterances. Returns (elapsed, admission) seconds,
        max over ranks. The voice state is precomputed: ONE voice shared by all rows (they read its
        KV prefix, KvStore::pre), or with distinct_voices a voice of its own per row (B distinct
        125-frame prompts: every row reads its own 6-MB prefix)."""
        if distinct_voices:
            voices = [eng.voice_from_prompt(synth_prompt(seed=100 + b)) for b in range(B)]
        else:
            voices = [eng.voice_from_prompt(synth_prompt())] * B

        def admit(round_id, n_frames):  # batched admission (ptts_slots_open): one shared text-prefill pass
            eng.open_many(list(range(B)), voices, [text_ids(b) for b in range(B)],
                          [params(round_id, b, n_frames) for b in range(B)])

        def run_calls(n_frames):
            """n_frames step calls (+ one when the admission starts a call late), then frame_lag()
            flush calls: they decode and deliver the frames already computed without running front
            parts for rows that have all finished (ptts_flush_async; a frame arrives lag calls late)"""
            lag, delay = eng.frame_lag()
            for _ in range(n_frames + delay):
                eng.step_async(B)
            for _ in range(lag):
                eng.flush_async(B) if pipeline and not args.no_flush else eng.step_async(B)

        # warmup: a short job on the same rows (graph capture, caches), then the rows are re-admitted
        admit(0, max(1, W))
        run_calls(max(1, W))
        eng.sync()
        barrier()
        eng.sync()
        job_s = []
        t0 = time.perf_counter()
        admit(1, K)
        eng.sync()
        admit_s = time.perf_counter() - t0  # one admission, alone (the later ones overlap, below)
        tj = t0
        for j in range(jobs):
            run_calls(K)  # the K frames, then the calls that drain the last one
            if j + 1 < jobs and not args.no_overlap_admission:
                # the next job's admission is issued now: its voice-KV copy and text prefill queue
                # behind this job's last front part and run beside its last back passes (the
                # engine resets the back part's slot state only after those, ptts_slots_open)
                admit(2 + j, K)
            r = eng.fetch(B)  # the last frame of every row (waits for this job's last back pass)
            assert r.valid.all() and r.last.all(), "bench produced invalid frames"
            assert np.isfinite(r.pcm).all(), "bench produced non-finite PCM"
            if j + 1 < jobs and args.no_overlap_admission:
                eng.sync()
                admit(2 + j, K)
            t = time.perf_counter()
            job_s.append(t - tj)
            tj = t
        t1 = time.perf_counter()
        barrier()
        elapsed = t1 - t0
        if dist is not None:
            elapsed, admit_s, *job_s = max_over_ranks(dist, [elapsed, admit_s, *job_s], dev)
        return elapsed, admit_s, job_s

    def pcm_sample(e, n_frames=24):
        """Every row's PCM, latents and EOS logits of n_frames frames at temp 0 (no EOS) from the
        bench's voice and texts: ([rows][frames][1920], [rows][frames][32], [rows][frames]) (the
        reduced-precision variants' accuracy against this engine's f32 outputs)."""
        voice = e.voice_from_prompt(synth_prompt())
        e.open_many(list(range(B)), [voice] * B, [text_ids(b) for b in range(B)],
                    [pt.GenerationParams(temp=0.0, eos_threshold=float("inf"), max_frames=n_frames, seed=b + 1)
                     for b in range(B)])
        out, lat, eos = [[] for _ in range(B)], [[] for _ in range(B)], [[] for _ in range(B)]
        for _ in range(n_frames + sum(e.frame_lag())):
            r = e.step(B)
            for b in range(B):
                if r.valid[b]:
                    out[b].append(r.pcm[b].copy())
                    lat[b].append(r.latents[b].copy())
                    eos[b].append(float(r.eos_logits[b]))
        assert all(len(o) == n_frames for o in out)
        return np.asarray(out, np.float64), np.asarray(lat, np.float64), np.asarray(eos, np.float64)

    def snr_rows(ref, x):
        """Per-row SNR (dB) of x against ref over all frames and channels of the row."""
        err = ((x - ref) ** 2).reshape(ref.shape[0], -1).sum(-1)
        return 10 * np.log10((ref ** 2).reshape(ref.shape[0], -1).sum(-1) / np.maximum(err, 1e-30))

    def accuracy_vs_f32(sample, ref):
        """A variant's accuracy against the f32 engine on the same 24-frame temp-0 sample: latent and
        PCM SNR (per row: min / median), EOS-logit error, and stop-frame agreement — per row, for
        thresholds at the f32 run's EOS-logit quartiles, the first frame above each (the reference's
        stop rule, tts_model.rs:1055-1063) on both engines (tests/test_fp8.py's measure)."""
        pcm, lat, eos = sample
        rpcm, rlat, reos = ref
        ls, ps = snr_rows(rlat, lat), snr_rows(rpcm, pcm)
        diffs = []
        for b in range(reos.shape[0]):
            for thr in np.quantile(reos[b], [0.25, 0.5, 0.75]):
                def stop(tr):
                    above = np.nonzero(tr > thr)[0]
                    return int(above[0]) if above.size else tr.size
                diffs.append(abs(stop(reos[b]) - stop(eos[b])))
        diffs = np.asarray(diffs)
        return {"latent_snr_db": {"min": round(float(ls.min()), 2), "median": round(float(np.median(ls)), 2)},
                "pcm_snr_db": {"min": round(float(ps.min()), 2), "median": round(float(np.median(ps)), 2)},
                "eos_logit_abs_err_max": round(float(np.abs(eos - reos).max()), 4),
                "stop_frame_same": round(float(np.mean(diffs == 0)), 3),
                "stop_frame_within_1": round(float(np.mean(diffs <= 1)), 3),
                "sample": f"{B} rows x {rpcm.shape[1]} frames, temp 0, bench voice and texts, against the f32 engine"}

    elapsed, admit_s, job_s = timed_job(eng)
    steps = jobs * K

    audio_sec = world * jobs * B * K * 1920 / 24000.0
    value = audio_sec / elapsed
    job_vals = sorted(world * B * K * 1920 / 24000.0 / t for t in job_s)
    per_job = {"jobs": jobs, "median": round(float(np.median(job_vals)), 2), "min": round(job_vals[0], 2),
               "max": round(job_vals[-1], 2)}

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return

    # ---- p50 first-chunk latency (config 2): text prefill + 1 step, voice precomputed
    p50 = None
    if not args.no_latency:
        e1 = pt.Engine(device=local_rank, max_slots=1, max_ctx=PROMPT_FRAMES + TEXT_TOKENS + 16, seed=0x5EED)
        v1 = e1.voice_from_prompt(synth_prompt())
        lat = []
        for i in range(55):
            t = time.perf_counter()
            e1.open(0, v1, text_ids(0), pt.GenerationParams(temp=0.7, eos_threshold=float("inf"), max_frames=4,
                                                             seed=i + 1))
            rr = e1.step(1)
            lat.append(time.perf_counter() - t)
            assert rr.valid[0]
        p50 = float(np.median(lat[5:]) * 1000.0)
        e1.close()

    # ---- configs[4] variants: the same job on an engine with the reference's int8 weight
    # quantization of the FlowLM (quantize.rs; its step GEMMs stream int8 codes), and with the
    # large FlowLM step GEMMs as fp8 W8A8 (accuracy-gated against the f32 oracle, tests/test_fp8.py).
    # Reported beside `value`, never as it (different numerics from the f32 reference).
    quant = fp8 = bf16 = None
    ref_sample = pcm_sample(eng) if not args.no_quant_variant and world == 1 and not selftest else None
    # the same job with B distinct voices: every row reads its own 125-frame prefix (6 MB of KV)
    # instead of the bench's one shared voice; the headline's shared-prefix benefit, made visible
    distinct = None
    if not args.no_distinct_voices and world == 1:
        d_el, d_ad, _ = timed_job(eng, distinct_voices=True)
        distinct = {"value": round(jobs * B * K * 1920 / 24000.0 / d_el, 2), "unit": "audio-sec/wall-sec",
                    "ms_per_step": round(1000.0 * d_el / steps, 4),
                    "steady_ms_per_step": round(1000.0 * (d_el - d_ad) / steps, 4),
                    "voices": f"{B} distinct {PROMPT_FRAMES}-frame prompts (one per row)",
                    "front_bytes_per_step": round(front_bytes(B, K, distinct_voices=B))}
    # ---- dominant kernel: time every op of the step plan on the engine stream (HIP events), with
    # the rows at the job's midpoint (context prompt + text + K/2, the job's mean: what the step's
    # attention ops read on average), on the bench's own shared voice. Last use of this engine:
    # the isolated replays rewrite slot state of the rows in flight
    roof, top, sum_ops_ms = None, None, None
    if not args.no_op_times:
        v_mid = eng.voice_from_prompt(synth_prompt())
        eng.open_many(list(range(B)), [v_mid] * B, [text_ids(b) for b in range(B)],
                      [params(0, b, K) for b in range(B)])
        for _ in range(K // 2 + eng.frame_lag()[1]):
            eng.step_async(B)
        eng.sync()
        plan = eng.plan(B)
        seen, per_op = set(), []
        for name, fl, by in plan:
            if name in seen:
                continue
            seen.add(name)
            us = eng.time_kernel(B, name, reps=20)
            per_op.append((us, name, fl, by))
        per_op.sort(reverse=True)
        # the dominant op is the LONGEST IN-STEP launch of the measured configuration (committed
        # kernel trace of this bench, profiles/op_stats.csv), where front and back share every CU;
        # the ops' isolated HIP-event times rank differently (in-step inflation differs per op).
        # Without a trace covering the plan, the longest isolated op stands in.
        ins = measured_in_step_all()
        alone = {n: (u, fl_, by_) for u, n, fl_, by_ in per_op}
        if ins and all(n in ins for n in alone):
            name = max(alone, key=lambda n: ins[n])
        else:
            name = per_op[0][1]
        us, fl, by = alone[name]
        intensity = fl / by if by else 0.0
        ridge = F32_PEAK_TFLOPS * 1e12 / (HBM_PEAK_GBS * 1e9)
        if by and intensity < ridge:
            roof = {"bound": "hbm", "achieved": round(by / (us * 1e-6) / 1e9, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s"}
        else:
            roof = {"bound": "mfma", "achieved": round(fl / (us * 1e-6) / 1e12, 2), "peak": F32_PEAK_TFLOPS,
                    "unit": "TFLOP/s"}
        roof["frac"] = round(roof["achieved"] / roof["peak"], 4)
        roof["traffic"], roof["traffic_source"] = measured_traffic(name)
        mf = measured_mfma().get(name)
        roof["rocprof_mfma_busy_frac"] = mf["util_peak_clock"] if mf else None
        roof["kernel"] = name
        # `achieved` / `frac` / `avg_us`: the op INSIDE the timed step, where the front and back parts
        # share every CU (committed rocprof trace of this bench, profiles/op_stats.csv); the same op
        # replayed alone on the engine stream (HIP events, live in this run) is `*_alone`
        roof["avg_us_alone"] = round(us, 2)
        roof["achieved_alone"] = roof["achieved"]
        roof["frac_alone"] = roof["frac"]
        roof["avg_us"] = roof["avg_us_alone"]
        roof["duration_source"] = "HIP events, op replayed alone (no committed in-step trace for it)"
        ius = measured_in_step(name)
        if ius:
            ach = by / (ius * 1e-6) / 1e9 if roof["unit"] == "GB/s" else fl / (ius * 1e-6) / 1e12
            roof["avg_us"] = round(ius, 2)
            roof["achieved"] = round(ach, 2 if roof["unit"] != "GB/s" else 1)
            roof["frac"] = round(ach / roof["peak"], 4)
            roof["duration_source"] = ("in-step average of its launches: profiles/op_stats.csv (rocprofv3 "
                                       "--kernel-trace of bench.py, tools/prof_ops.py piped)")
        roof["algorithmic_bytes"] = by
        roof["algorithmic_flops"] = fl
        roof["kernel_aggregate"] = kernel_aggregates()
        # top_ops: the step's longest launches IN STEP (what the step pays for), each with its
        # isolated time and the in-step / alone inflation
        if ins and all(n in ins for n in alone):
            ranked = sorted(alone, key=lambda n: -ins[n])[:8]
            top = [{"op": n, "avg_us_in_step": round(ins[n], 2), "avg_us_alone": round(alone[n][0], 2),
                    "inflation": round(ins[n] / alone[n][0], 3)} for n in ranked]
        else:
            top = [{"op": n, "avg_us_alone": round(u, 2)} for u, n, _, _ in per_op[:8]]
        sum_ops_ms = round(sum(u for u, _, _, _ in per_op) / 1000.0, 3)
        roof["phases"] = phase_rooflines(per_op, plan, B, K, back_frames)
        roof["step"] = step_roofline(plan, B, K, back_frames, 1e6 * (elapsed - admit_s) / steps)
        if args.ops_out:
            with open(args.ops_out, "w") as f:
                json.dump({"n_rows": B, "plan": [n for n, _, _ in plan],
                           "ops": [{"op": n, "avg_us": u, "flops": fl_, "bytes": by_} for u, n, fl_, by_ in per_op]},
                          f, indent=1)
    elif args.ops_out and not selftest:
        with open(args.ops_out, "w") as f:
            json.dump({"n_rows": B, "plan": [n for n, _, _ in eng.plan(B)], "ops": []}, f, indent=1)

    eng.close()  # one engine on the GPU at a time
    if not args.no_quant_variant and world == 1:
        eq = pt.Engine(device=local_rank, max_slots=B, max_ctx=max_ctx, lsd_decode_steps=1, seed=0x5EED,
                       pipeline=pipeline, back_frames=back_frames, weight_quant=pt.QUANT_FLOW_LM)
        q_el, q_ad, _ = timed_job(eq)
        q_acc = accuracy_vs_f32(pcm_sample(eq), ref_sample)
        quant = {"value": round(jobs * B * K * 1920 / 24000.0 / q_el, 2), "unit": "audio-sec/wall-sec",
                 "ms_per_step": round(1000.0 * q_el / steps, 4),
                 "steady_ms_per_step": round(1000.0 * (q_el - q_ad) / steps, 4),
                 "weight_quant": "flow_lm int8 (quantize.rs QuantizeConfig::default, per-tensor symmetric; equals "
                                 "the quantized oracle at the f32 gates, tests/test_quantize.py)",
                 "int8_matrices": eq.int8_matrices, "accuracy_vs_f32": q_acc}
        eq.close()
        ef = pt.Engine(device=local_rank, max_slots=B, max_ctx=max_ctx, lsd_decode_steps=1, seed=0x5EED,
                       pipeline=pipeline, back_frames=back_frames, fp8_gemm=True)
        f_el, f_ad, _ = timed_job(ef)
        f_acc = accuracy_vs_f32(pcm_sample(ef), ref_sample)
        fp8 = {"value": round(jobs * B * K * 1920 / 24000.0 / f_el, 2), "unit": "audio-sec/wall-sec",
               "ms_per_step": round(1000.0 * f_el / steps, 4),
               "steady_ms_per_step": round(1000.0 * (f_el - f_ad) / steps, 4),
               "gemm": "fp8 e4m3 W8A8 on v_mfma_f32_32x32x16_fp8_fp8 (row-scaled weights, per-slice "
                       "activation scales), FlowLM qkv/linear1/linear2/adaLN",
               "numerics": f"reduced precision, NOT the reference's: latent SNR "
                           f"{f_acc['latent_snr_db']['min']:.1f} dB (worst row) against f32",
               "fp8_matrices": ef.fp8_matrices, "accuracy_vs_f32": f_acc}
        ef.close()
        # the Mimi decode (back part) on bf16 MFMA: the same job, and its PCM against the f32
        # engine's (= the f32 oracle within 1e-7, tests/test_gpu_bench_shape.py) on a 24-frame sample
        eb = pt.Engine(device=local_rank, max_slots=B, max_ctx=max_ctx, lsd_decode_steps=1, seed=0x5EED,
                       pipeline=pipeline, back_frames=back_frames, back_bf16=True)
        b_el, b_ad, _ = timed_job(eb)
        bp = pcm_sample(eb)[0]
        eb.close()
        ref_pcm = ref_sample[0]
        err = ((bp - ref_pcm) ** 2).sum(-1)
        snr = 10 * np.log10((ref_pcm ** 2).sum(-1) / np.maximum(err, 1e-30))
        bf16 = {"value": round(jobs * B * K * 1920 / 24000.0 / b_el, 2), "unit": "audio-sec/wall-sec",
                "ms_per_step": round(1000.0 * b_el / steps, 4),
                "steady_ms_per_step": round(1000.0 * (b_el - b_ad) / steps, 4),
                "mfma": "Mimi decoder transformer GEMMs + SEANet decoder convs on v_mfma_f32_32x32x16_bf16 "
                        "(operands rounded to bf16, f32 accumulation); FlowLM, attention, final conv f32",
                "pcm_snr_db_vs_f32": {"min": round(float(snr.min()), 2), "median": round(float(np.median(snr)), 2),
                                      "frames": int(snr.size), "gate_min": 30.0},
                "latents_eos_stop_frames": "unchanged (f32 FlowLM; the back part does not feed it): "
                                           "tests/test_gpu_bf16.py"}

    # ---- configs[4]'s voice-cloning leg and the reference's text-driven generation benchmark
    voice_bench = text_bench = None
    if not args.no_voice_bench and world == 1:
        voice_bench = {"gpu": voice_state_bench(pt, local_rank)}
        if not args.no_cpu_baseline:
            voice_bench["cpu_baseline"] = cpu_voice_leg(args.cpu_procs)
    if not args.no_text_bench and world == 1:
        text_bench = text_e2e_bench(pt, local_rank)

    # ---- CPU baseline: the oracle (C restatement of the reference algorithm) on the host cores,
    # the same 125-frame job per utterance (oracle/cpu_baseline.py, a child process)
    cpu = None
    if not args.no_cpu_baseline and world == 1:
        cpu = cpu_baseline_leg(args.cpu_procs)

    # ---- what was measured: the product library built from these sources, no PTTS_* knobs
    tuned = {k: v for k, v in os.environ.items() if k.startswith("PTTS_")}
    build = None
    if not selftest:
        build = pt.build_id()
        if build != pt.source_build_id():
            tuned["build_id"] = f"{build} (sources: {pt.source_build_id()})"
    data = ("launcher selftest (CPU stand-in engine, nothing computed)" if selftest else
            f"PROFILING RUN ({K}-frame utterances, not configs[2])" if args.profile_frames > 0 else
            "synthetic (seeded weights and prompts; real checkpoints are gated offline)")
    if tuned:
        data = "NOT A PRODUCT RUN (PTTS_* knobs or a non-matching build; see tuned): " + data

    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "audio-sec/wall-sec",
        "n_gpus": world,
        "steps": steps,
        "steps_requested": args.steps,
        "warmup": W,
        "ms_per_step": round(1000.0 * elapsed / steps, 4),
        "admit_ms": round(1000.0 * admit_s, 3),  # the first job's admission, alone (synchronised)
        # per frame, drain calls included, without the first job's admission (the only one that does
        # not overlap the previous job's last back passes; the later ones are issued right after the
        # previous job's drain calls and run beside them, so their wall cost is inside the steps)
        "steady_ms_per_step": round(1000.0 * (elapsed - admit_s) / steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": data,
        "config": {"workload": f"b6369a24 batch={B} concurrent 10 s utterances per GPU (125 frames, voice prompt "
                               f"{PROMPT_FRAMES} frames, {TEXT_TOKENS} text tokens), lsd_decode_steps=1 "
                               "(BASELINE configs[2])",
                   "global_batch": B * world, "utterance_frames": K, "jobs": jobs, "prompt_frames": PROMPT_FRAMES,
                   "text_tokens": TEXT_TOKENS, "temp": 0.7, "parallelism": f"replicas x{world}",
                   "stepping": (f"pipelined, {back_frames} frames per Mimi decode pass (overlapping the "
                                "FlowLM steps of the next frames)" if back_frames > 1 else
                                "pipelined (Mimi decode of frame k overlaps FlowLM step k+1)") if pipeline
                   else "sequential",
                   "pcm_to_host": "every frame, async D2H into pinned memory inside the step graphs"},
        "per_job": per_job,
        "build_id": build,
        "tuned": tuned or None,
        "p50_first_chunk_ms": None if p50 is None else round(p50, 3),
        "int8_flowlm_variant": quant,
        "fp8_flowlm_variant": fp8,
        "bf16_back_variant": bf16,
        "distinct_voices_variant": distinct,
        "voice_encode_ms": voice_bench,
        "text_generate": text_bench,
        "roofline": roof,
        "cpu_baseline": cpu,
        "top_ops": top,
        "sum_op_ms": sum_ops_ms,
    }
    print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
