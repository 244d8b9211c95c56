"""bf16 back part (ptts_engine_config.back_bf16): the Mimi decoder transformer GEMMs and the SEANet
decoder convs on v_mfma_f32_32x32x16_bf16 (operands rounded to bf16, f32 accumulation), a variant
beside the f32 path (the reference's own quantization scope includes Mimi,
quantize.rs:1-219). Not a reference numeric, so gated on accuracy against the f32 oracle:
  * latents and EOS logits: the f32 gates (LAT_TOL) - the back part does not feed the FlowLM;
  * PCM: SNR >= 30 dB per frame and row against the oracle's f32 PCM;
  * stop frames with EOS on: identical to the oracle's rule (tts_model.rs:1055-1063).
It applies at >= 16 rows (the MFMA-bound shapes): 16 rows here, frame pairs as in the bench."""

import numpy as np
import pytest
from conftest import LAT_TOL, load_golden

pytestmark = pytest.mark.gpu

SNR_GATE_DB = 30.0


def snr_db(ref, x):
    ref, x = np.asarray(ref, np.float64), np.asarray(x, np.float64)
    return 10 * np.log10(np.sum(ref * ref) / max(np.sum((x - ref) ** 2), 1e-30))


@pytest.mark.parametrize("back_frames", [1, 2, 4])
def test_bf16_back_accuracy_and_stop_frames(oracle, back_frames):
    import pocket_tts_amd as pt

    d = load_golden("e2e_lsd1.safetensors")
    rng = np.random.default_rng(21)
    B, n_frames = 16, 10
    eng = pt.Engine(device=0, max_slots=B, max_ctx=128, lsd_decode_steps=1, seed=0x5EED, pipeline=True,
                    back_frames=back_frames, back_bf16=True)
    try:
        orc, lat, got, vs, ids_l, want = {}, {}, {}, [], [], {}
        for b in range(B):
            F = 4 + b % 7
            prompt = (d["prompt"][:F] * (1.0 + 0.02 * b)).astype(np.float32)
            ids = rng.integers(0, 4000, size=3 + b % 5).astype(np.int32)
            vs.append(eng.voice_from_prompt(prompt))
            ids_l.append(ids)
            s = oracle.new_state(128)
            s.prefill(prompt)
            s.prefill_tokens(ids)
            orc[b], lat[b], got[b] = s, None, 0
        # EOS on for half the rows (threshold inside the golden logits' range: rows stop early,
        # frames_after_eos 2), off for the other half
        thr = [-0.45 if b % 2 else float("inf") for b in range(B)]
        eng.open_many(list(range(B)), vs, ids_l,
                      [pt.GenerationParams(temp=0.0, eos_threshold=thr[b], frames_after_eos=2, max_frames=n_frames,
                                           seed=1) for b in range(B)])
        # the oracle's stop rule per row (its own EOS logits)
        snrs, done = [], set()
        for _ in range(n_frames + sum(eng.frame_lag()) + 1):  # a frame arrives frame_lag() calls late
            r = eng.step(B)
            for b in range(B):
                if not r.valid[b]:
                    continue
                assert b not in done, b
                o = orc[b].step(lat[b])
                lat[b] = o["latent"]
                got[b] += 1
                assert abs(r.eos_logits[b] - o["eos_logit"]) <= LAT_TOL
                np.testing.assert_allclose(r.latents[b], o["latent"], atol=LAT_TOL)
                snrs.append(snr_db(o["pcm"], r.pcm[b]))
                if o["eos_logit"] > thr[b] and b not in want:
                    want[b] = got[b] - 1 + 2  # eos step + frames_after_eos
                expect_last = got[b] == n_frames or (b in want and got[b] - 1 >= want[b])
                assert bool(r.last[b]) == expect_last, (b, got[b])
                if r.last[b]:
                    done.add(b)
        assert done == set(range(B))
        assert any(got[b] < n_frames for b in range(B)), "EOS stopped no row"
        print(f"back_frames={back_frames}: PCM SNR vs f32 oracle min {min(snrs):.1f} dB, "
              f"median {np.median(snrs):.1f} dB over {len(snrs)} frames")
        assert min(snrs) >= SNR_GATE_DB
    finally:
        eng.close()
