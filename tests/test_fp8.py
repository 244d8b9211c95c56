"""fp8 W8A8 GEMM path (BASELINE configs[4] "fp8 MFMA GEMM path").

Pinning. The reference has no fp8 arithmetic (quantize.rs is a simulated int8 grid and its
load_quantized is a placeholder, tts_model.rs:150-179), so there are no reference outputs to
match: parity is unpinned by construction and this path is gated on ACCURACY against the f32
oracle instead, like the reference's own quantization tests gate on SNR (quantize.rs:179-201).

What runs in fp8 (ptts_engine_config.fp8_gemm = 1): the large FlowLM step GEMMs (per layer
in_proj, linear1, linear2, and the flow head's fused adaLN matrix: 19 matrices). Weights are OCP
e4m3 codes with one scale per output row (max|w| / 448); activations are quantized in-kernel
with one scale per (row, split-K slice); v_mfma_f32_32x32x16_fp8_fp8 accumulates in f32. Every
other op stays f32.

The CPU tests restate the e4m3 encoding (round to nearest even, 3 mantissa bits, max 448) and
the kernel's W8A8 arithmetic in numpy, and record the error model the GPU gates are set from."""

import numpy as np
import pytest
from conftest import load_golden

import _oracle  # noqa: F401  (builds/loads the oracle for the GPU tests)

N_FP8_MATRICES = 6 * 3 + 1  # qkv, linear1, linear2 per FlowLM layer + the head's adaLN


def e4m3(x):
    """OCP e4m3fn value nearest to x (round half to even), saturating at +-448 (the kernels
    scale every operand into [-448, 448] first, so saturation never changes a value)."""
    x = np.asarray(x, np.float64)
    a = np.minimum(np.abs(x), 448.0)
    e = np.floor(np.log2(np.maximum(a, 2.0 ** -9)))
    e = np.maximum(e, -6.0)  # subnormals: spacing 2^-9 below 2^-6
    step = 2.0 ** (e - 3)
    q = np.round(a / step) * step  # numpy rounds half to even
    return (np.sign(x) * np.minimum(q, 448.0)).astype(np.float32)


def w8a8_gemm(X, W, slices):
    """k_gemm_fp8's arithmetic: W rows scaled by max|w|/448, X rows per K slice by max|x|/448,
    products of codes summed in f64 (f32 in the MFMA), slices summed."""
    X = np.asarray(X, np.float64)
    W = np.asarray(W, np.float64)
    sw = np.abs(W).max(axis=1) / 448.0
    sw[sw == 0] = 1.0
    Wq = e4m3(W / sw[:, None]).astype(np.float64)
    out = np.zeros((X.shape[0], W.shape[0]))
    for k0, k1 in slices:
        xs = X[:, k0:k1]
        sa = np.abs(xs).max(axis=1) / 448.0
        inv = np.where(sa > 0, 1.0 / np.where(sa > 0, sa, 1.0), 0.0)
        Xq = e4m3(xs * inv[:, None]).astype(np.float64)
        out += (Xq @ Wq[:, k0:k1].T) * sa[:, None] * sw[None, :]
    return out


def snr_db(ref, x):
    ref = np.asarray(ref, np.float64)
    return float(10 * np.log10(np.sum(ref ** 2) / max(np.sum((np.asarray(x, np.float64) - ref) ** 2), 1e-300)))


def test_e4m3_grid():
    # exactly representable values round-trip; halfway cases go to the even mantissa
    for v in [0.0, 1.0, 1.125, 448.0, -448.0, 2.0 ** -6, 2.0 ** -9, 3.5, 240.0]:
        assert e4m3(v) == np.float32(v)
    assert e4m3(1.0625) == np.float32(1.0)  # halfway between 1.0 and 1.125 -> even (1.0)
    assert e4m3(1.1875) == np.float32(1.25)  # halfway between 1.125 and 1.25 -> even (1.25)
    assert e4m3(500.0) == np.float32(448.0)
    g = e4m3(np.linspace(-448, 448, 20001))
    assert np.unique(g).size <= 253  # 126 positive finite magnitudes, their negatives, and 0


def test_w8a8_error_model():
    """Relative error of one W8A8 GEMM at FlowLM shapes: ~28-30 dB SNR (e4m3 has 3 mantissa
    bits: a uniform rounding error of 2^-4 relative, averaged over K products)."""
    rng = np.random.default_rng(0)
    for M, N, K, S in [(32, 3072, 1024, 8), (32, 1024, 4096, 16), (32, 4096, 1024, 4)]:
        X = rng.standard_normal((M, K)).astype(np.float32)
        W = (rng.uniform(-1, 1, (N // 8, K)) / np.sqrt(K)).astype(np.float32)
        ref = X.astype(np.float64) @ W.T.astype(np.float64)
        ks = K // S
        got = w8a8_gemm(X, W, [(z * ks, (z + 1) * ks) for z in range(S)])
        assert snr_db(ref, got) > 24.0, (M, N, K, snr_db(ref, got))


# ---------------------------------------------------------------- GPU: fp8 engine vs f32 oracle
# Gates from the measured error: per-step latents and PCM of a free-running
# temp-0 generation against the f32 oracle, first 8 frames.
LATENT_SNR_DB = 15.0  # measured 18.7 (B = 1) and 19.2 (worst of 32 rows)
PCM_SNR_DB = 30.0  # measured 49.9
EOS_ABS = 0.5


def _oracle_state(o, prompt, ids):
    s = o.new_state(256)
    s.prefill(prompt)
    s.prefill_tokens(ids)
    return s


@pytest.mark.gpu
def test_gpu_fp8_engine_accuracy_vs_f32_oracle():
    import pocket_tts_amd as pt
    from _oracle import Oracle

    d = load_golden("e2e_lsd1.safetensors")
    steps = 8
    eng = pt.Engine(device=0, max_slots=1, max_ctx=256, seed=0x5EED, fp8_gemm=True)
    try:
        assert eng.fp8_matrices == N_FP8_MATRICES
        eng.open(0, eng.voice_from_prompt(d["prompt"]), d["text_ids"],
                 pt.GenerationParams(temp=0.0, eos_threshold=float("inf"), max_frames=steps))
        s = _oracle_state(Oracle(0x5EED), d["prompt"], d["text_ids"])
        lat = None
        lats, rlats, pcms, rpcms = [], [], [], []
        for i in range(steps):
            r = eng.step(1)
            ref = s.step(lat)
            lat = ref["latent"]
            assert r.valid[0] and np.isfinite(r.pcm[0]).all()
            assert abs(r.eos_logits[0] - ref["eos_logit"]) <= EOS_ABS, (i, r.eos_logits[0], ref["eos_logit"])
            lats.append(r.latents[0].copy())
            rlats.append(ref["latent"])
            pcms.append(r.pcm[0].copy())
            rpcms.append(ref["pcm"])
        ls, ps = snr_db(np.stack(rlats), np.stack(lats)), snr_db(np.stack(rpcms), np.stack(pcms))
        print(f"fp8 vs f32 oracle, {steps} frames: latent SNR {ls:.1f} dB, PCM SNR {ps:.1f} dB")
        assert ls >= LATENT_SNR_DB and ps >= PCM_SNR_DB, (ls, ps)
    finally:
        eng.close()


@pytest.mark.gpu
def test_gpu_fp8_batched_pipelined():
    """B = 32 rows (the bench shape: 32-row tiles, split-K slices <= 512) under pipelined graph
    stepping: every row within the gate of its own f32 oracle run; rows are independent."""
    import pocket_tts_amd as pt
    from _oracle import Oracle

    d = load_golden("e2e_lsd1.safetensors")
    rng = np.random.default_rng(9)
    B, steps = 32, 4
    eng = pt.Engine(device=0, max_slots=B, max_ctx=256, seed=0x5EED, fp8_gemm=True, pipeline=True)
    o = Oracle(0x5EED)
    try:
        states = []
        for b in range(B):
            prompt = (d["prompt"][: 4 + (b % 5)] * (1 + 0.02 * b)).astype(np.float32)
            ids = rng.integers(0, 4000, size=3 + b % 4).astype(np.int32)
            eng.open(b, eng.voice_from_prompt(prompt), ids,
                     pt.GenerationParams(temp=0.0, eos_threshold=float("inf"), max_frames=steps))
            states.append(_oracle_state(o, prompt, ids))
        lats = [None] * B
        got = {b: ([], []) for b in range(B)}
        for call in range(steps + 1):
            r = eng.step(B)
            if call == 0:
                assert not r.valid.any()
                continue
            for b in range(B):
                ref = states[b].step(lats[b])
                lats[b] = ref["latent"]
                assert r.valid[b]
                got[b][0].append(r.latents[b].copy())
                got[b][1].append(ref["latent"])
        worst = min(snr_db(np.stack(g[1]), np.stack(g[0])) for g in got.values())
        print(f"fp8 B={B}: worst-row latent SNR {worst:.1f} dB")
        assert worst >= LATENT_SNR_DB, worst
    finally:
        eng.close()


@pytest.mark.gpu
def test_gpu_fp8_config_errors():
    import pocket_tts_amd as pt

    with pytest.raises(pt.PocketTTSError, match="exclusive"):
        pt.Engine(device=0, max_slots=1, max_ctx=64, fp8_gemm=True, weight_quant=1)
    eng = pt.Engine(device=0, max_slots=1, max_ctx=64)
    try:
        assert eng.fp8_matrices == 0
    finally:
        eng.close()


@pytest.mark.gpu
def test_gpu_fp8_eos_frame_count_agreement():
    """Frame-count agreement (where each utterance would stop) of the fp8 engine against the f32
    engine: 32 rows, temp 0, 24 frames with the EOS rule off, so both runs see the same
    prompts; then, for every row and for each threshold between the f32 run's EOS-logit
    quartiles, the first frame whose logit exceeds it (tts_model.rs:1055-1063) is compared.
    Measured, not matched: fp8 has no reference numerics (the f32 engine's own EOS rule is
    pinned by test_eos_termination_rule)."""
    import json

    import pocket_tts_amd as pt

    d = load_golden("e2e_lsd1.safetensors")
    rng = np.random.default_rng(11)
    B, steps = 32, 24
    rows = []
    for b in range(B):
        prompt = (d["prompt"][: 4 + (b % 5)] * (1 + 0.02 * b)).astype(np.float32)
        rows.append((prompt, rng.integers(0, 4000, size=3 + b % 4).astype(np.int32)))
    logits = {}
    for fp8 in (False, True):
        eng = pt.Engine(device=0, max_slots=B, max_ctx=256, seed=0x5EED, fp8_gemm=fp8)
        try:
            for b, (prompt, ids) in enumerate(rows):
                eng.open(b, eng.voice_from_prompt(prompt), ids,
                         pt.GenerationParams(temp=0.0, eos_threshold=float("inf"), max_frames=steps))
            tr = []
            for _ in range(steps):
                r = eng.step(B)
                assert r.valid.all() and np.isfinite(r.eos_logits).all()
                tr.append(r.eos_logits.copy())
            logits[fp8] = np.stack(tr, axis=1)  # [B][steps]
        finally:
            eng.close()
    f32, f8 = logits[False], logits[True]
    diffs, same, total = [], 0, 0
    for b in range(B):
        for thr in np.quantile(f32[b], [0.25, 0.5, 0.75]):
            def stop(tr):
                above = np.nonzero(tr > thr)[0]
                return int(above[0]) if above.size else steps
            d32, d8 = stop(f32[b]), stop(f8[b])
            diffs.append(abs(d32 - d8))
            same += d32 == d8
            total += 1
    diffs = np.asarray(diffs)
    summary = {"rows": B, "thresholds_per_row": 3, "same_stop_frame": round(same / total, 3),
               "within_1_frame": round(float(np.mean(diffs <= 1)), 3),
               "median_abs_frames": float(np.median(diffs)), "max_abs_frames": int(diffs.max()),
               "eos_logit_abs_err_max": round(float(np.abs(f32 - f8).max()), 4),
               "eos_logit_spread_f32": round(float(np.median(f32.max(1) - f32.min(1))), 4)}
    print("fp8 frame-count agreement:", json.dumps(summary))
    # gates set from the measurement
    assert np.abs(f32 - f8).max() <= EOS_ABS
    assert summary["within_1_frame"] >= 0.5, summary  # measured 0.77 (same frame 0.59, EOS |d| <= 0.17)


@pytest.mark.gpu
@pytest.mark.parametrize("pipeline,back_frames", [(False, 1), (True, 1), (True, 2)])
def test_gpu_fp8_matrices_stream_codes_in_every_stepping_mode(pipeline, back_frames):
    """every fp8 matrix must run W8A8 in every stepping mode. In single-frame pipelined
    stepping linear2 has no fused feed-forward and no {4, 128} register-resident tile; it used to
    land on the f32 register-resident GEMM there. The plan's algorithmic bytes state what each
    launch streams: one byte per weight on the fp8 path, four on an f32 one."""
    import pocket_tts_amd as pt

    B = 32
    eng = pt.Engine(device=0, max_slots=B, max_ctx=128, seed=0x5EED, fp8_gemm=True, pipeline=pipeline,
                    back_frames=back_frames)
    try:
        assert eng.fp8_matrices == N_FP8_MATRICES
        eng.open_many(list(range(B)), [eng.voice_from_prompt(np.zeros((4, 1024), np.float32))] * B,
                      [np.array([1, 2, 3], np.int32)] * B,
                      [pt.GenerationParams(temp=0.0, eos_threshold=float("inf"), max_frames=4)] * B)
        plan = {n: (fl, by) for n, fl, by in eng.plan(B)}
        weights = {"qkv_gemm": 3072 * 1024, "ff1_gemm": 4096 * 1024, "ff2_gemm": 1024 * 4096, "ffn": 2 * 4096 * 1024}
        seen = 0
        for name, (fl, by) in plan.items():
            kind = name.split(".")[-1]
            if name.startswith("flow.l") and kind in weights:
                # codes: 1 B per weight (+ activations and split-K slabs), f32: >= 4 B per weight
                assert by < 3.0 * weights[kind], (name, by)
                seen += 1
        assert plan["head.ada_gemm"][1] < 3.0 * 10240 * 512
        # per layer: qkv + (ffn | ff1 + ff2)
        assert seen >= 6 * 2, sorted(plan)
    finally:
        eng.close()
