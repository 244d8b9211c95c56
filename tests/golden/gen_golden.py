#!/usr/bin/env python3
"""Generate the golden parity fixtures from the reference's own Python modules.

RUN HERE ONLY (needs /root/reference, which does not exist on the GPU box).
The fixtures it writes (tests/golden/*.safetensors) are data: inputs and the
reference's outputs for them. The reference itself never ships.

Recipe:
  * stub the absent `beartype` package, import `python-reference/pocket_tts`;
  * build FlowLMModel / MimiModel from `config/b6369a24.yaml` without
    `TTSModel.load_model` (which downloads);
  * fill every parameter from the shared PRNG in `synth.py`;
  * "Candle semantics" switch: the Rust reference's
    FFN uses Candle's tanh-approximate GELU (`models/transformer.rs:85`), so
    `F.gelu` inside `modules/mimi_transformer.py:174` is swapped for the tanh
    form;
  * drive the loop the way `tts_model.rs:935-1071` does: voice prompt prefill
    (`tts_model.rs:580-599`), text prefill (`:958-964`), then per step
    FlowLM forward with empty text (`:1016-1030`), denorm + quantize
    (`:1033-1038`) and Mimi decode (`:1039-1045`), temperature 0.

Usage:  python tests/golden/gen_golden.py   (takes ~1 min on 8 cores)
"""

from __future__ import annotations

import os
import sys
import types
import typing
from functools import partial
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
import synth  # noqa: E402

REF = Path(os.environ.get("PTTS_REFERENCE", "/root/reference/python-reference"))
SEED = 0x5EED


def _import_reference():
    bt = types.ModuleType("beartype")
    bt.BeartypeConf = lambda **k: None
    claw = types.ModuleType("beartype.claw")
    claw.beartype_this_package = lambda **k: None
    btt = types.ModuleType("beartype.typing")
    btt.Callable = typing.Callable
    btt.Iterator = typing.Iterator
    bt.claw, bt.typing = claw, btt
    sys.modules.update({"beartype": bt, "beartype.claw": claw, "beartype.typing": btt})
    sys.path.insert(0, str(REF))
    import torch

    import pocket_tts.modules.mimi_transformer as mt

    shim = types.SimpleNamespace(**{k: getattr(torch.nn.functional, k) for k in dir(torch.nn.functional) if not k.startswith("__")})
    shim.gelu = lambda x: torch.nn.functional.gelu(x, approximate="tanh")
    mt.F = shim
    return torch


def build_models(torch):
    from pocket_tts.models.flow_lm import FlowLMModel
    from pocket_tts.models.mimi import MimiModel
    from pocket_tts.modules.dummy_quantizer import DummyQuantizer
    from pocket_tts.modules.mimi_transformer import ProjectedTransformer, StreamingTransformer
    from pocket_tts.modules.mlp import SimpleMLPAdaLN
    from pocket_tts.modules.seanet import SEANetDecoder, SEANetEncoder
    from pocket_tts.utils.config import load_config

    cfg = load_config(REF / "pocket_tts/config/b6369a24.yaml")
    flow_net = SimpleMLPAdaLN.from_pydantic_config(cfg.flow_lm, 32, 1024)
    tr = StreamingTransformer.from_pydantic_config(cfg.flow_lm.transformer)

    class Cond(torch.nn.Module):  # stands in for LUTConditioner (which downloads a tokenizer)
        def __init__(self):
            super().__init__()
            self.embed = torch.nn.Embedding(4001, 1024)

    flm = FlowLMModel(Cond(), flow_net, tr, dim=1024, ldim=32, dtype=torch.float32)
    m = cfg.mimi.model_dump()
    enc = SEANetEncoder(**m["seanet"])
    dec = SEANetDecoder(**m["seanet"])
    mimi = MimiModel(
        enc, dec, DummyQuantizer(**m["quantizer"]), channels=1, sample_rate=24000,
        frame_rate=12.5, encoder_frame_rate=24000 / enc.hop_length,
        encoder_transformer=ProjectedTransformer(**m["transformer"]),
        decoder_transformer=ProjectedTransformer(**m["transformer"]),
    )
    for prefix, mod in (("flow_lm.", flm), ("mimi.", mimi)):
        sd = mod.state_dict()
        for k, v in sd.items():
            t = synth.synth_tensor(SEED, prefix + k, tuple(v.shape))
            if t is not None:
                sd[k] = torch.from_numpy(t)
        mod.load_state_dict(sd, strict=True)
        mod.eval()
    speaker_proj = torch.from_numpy(synth.synth_tensor(SEED, "flow_lm.speaker_proj_weight", (1024, 512)))
    return flm, mimi, speaker_proj


def run_e2e(torch, flm, mimi, F, S, N, lsd_steps, tag, ids=None, eos_threshold=-4.0, frames_after_eos=None):
    """N frames at temp 0 from a synthetic F-frame voice prompt and S text ids (random unless
    `ids` is given). frames_after_eos set: the Rust segment's stop rule (tts_model.rs:1055-1063):
    the frame at eos_step + frames_after_eos is the last, N is max_gen_len."""
    from pocket_tts.modules.stateful_module import increment_steps, init_states

    prompt = synth.gaussian(1, f"{tag}/prompt", F * 1024, 0.11).reshape(F, 1024)
    if ids is None:
        ids = (synth.uniform01(2, f"{tag}/ids", S) * 4000).astype(np.int32)
    ids = np.asarray(ids, np.int32)
    S = ids.size
    eos_step = None
    caps = {}
    h1 = flm.out_norm.register_forward_hook(lambda m, i, o: caps.__setitem__("tout", o[:, -1].clone()))
    h2 = flm.out_eos.register_forward_hook(lambda m, i, o: caps.__setitem__("eos", o.clone()))
    out = {"prompt": prompt, "text_ids": ids}
    with torch.no_grad():
        state = init_states(flm, batch_size=1, sequence_length=1000)
        flm.transformer(torch.from_numpy(prompt)[None], state)
        increment_steps(flm, state, increment=F)
        emb = flm.conditioner.embed(torch.from_numpy(ids.astype(np.int64)))[None]
        flm.transformer(emb, state)
        increment_steps(flm, state, increment=S)
        mimi_state = init_states(mimi, batch_size=1, sequence_length=1000)
        backbone = torch.full((1, 1, 32), float("nan"))
        empty = torch.empty((1, 0, 1024))
        touts, eos, lats, pcms, quant, ups, trs = [], [], [], [], [], [], []
        for step in range(N):
            lat, is_eos = flm._sample_next_latent(backbone, empty, model_state=state, lsd_decode_steps=lsd_steps,
                                                  temp=0.0, noise_clamp=None, eos_threshold=eos_threshold)
            increment_steps(flm, state, increment=1)
            touts.append(caps["tout"][0].numpy().copy())
            eos.append(float(caps["eos"][0, 0]))
            lats.append(lat[0].numpy().copy())
            x = lat * flm.emb_std + flm.emb_mean
            q = mimi.quantizer(x[:, :, None])
            up = mimi.upsample(q, mimi_state)
            (tr_out,) = mimi.decoder_transformer(up, mimi_state)
            pcm = mimi.decoder(tr_out, mimi_state)
            increment_steps(mimi, mimi_state, increment=16)
            pcms.append(pcm[0, 0].numpy().copy())
            if step < 3:
                quant.append(q[0, :, 0].numpy().copy())
                ups.append(up[0].numpy().copy())
                trs.append(tr_out[0].numpy().copy())
            backbone = lat[:, None, :]
            if frames_after_eos is not None:
                if bool(is_eos) and eos_step is None:
                    eos_step = step
                if eos_step is not None and step >= eos_step + frames_after_eos:
                    break
    h1.remove()
    h2.remove()
    out.update(
        tout=np.stack(touts), eos_logit=np.array(eos, np.float32), latent=np.stack(lats),
        pcm=np.stack(pcms), quantized=np.stack(quant), after_upsample=np.stack(ups),
        after_decoder_transformer=np.stack(trs),
        meta=np.array([SEED, F, S, N, lsd_steps], np.int64),
    )
    if frames_after_eos is not None:
        out["stop"] = np.array([len(lats), -1 if eos_step is None else eos_step, frames_after_eos, N], np.int64)
        out["eos_threshold"] = np.array([eos_threshold], np.float32)
    return out


def run_encoder(torch, mimi, speaker_proj, n_frames, tag):
    """Voice cloning front half: PCM -> Mimi latent -> speaker projection (tts_model.py:258-262)."""
    pcm = synth.gaussian(3, f"{tag}/pcm", n_frames * 1920, 0.1)
    with torch.no_grad():
        x = torch.from_numpy(pcm)[None, None]
        emb = mimi.encoder(x, model_state=None)
        (tr,) = mimi.encoder_transformer(emb, model_state=None)
        lat = mimi._to_framerate(tr)
        cond = torch.nn.functional.linear(lat.transpose(-1, -2), speaker_proj)
    return {"pcm": pcm, "after_encoder": emb[0].numpy(), "after_encoder_transformer": tr[0].numpy(),
            "latent": lat[0].numpy(), "conditioning": cond[0].numpy(),
            "meta": np.array([SEED, n_frames], np.int64)}


def run_encoder_chunked(torch, mimi, speaker_proj, n_frames, chunk_frames, tag):
    """The Rust voice encode (tts_model.rs:520-541): PCM cut into chunks of `chunk_frames` frames,
    each pushed through `encode_to_latent(chunk, &mut model_state, 0)` with ONE carried state.
    Every chunk passes step=0, so the replicate-padded ConvDownsample1d re-pads from each chunk's
    first frame (conv.rs:116-123) instead of using its carried `previous`. Emulated with the
    reference's own Python streaming modules: one state from `init_states`, and the downsample
    conv's `first` flag raised before every chunk (conv.py:101-106)."""
    from pocket_tts.modules.stateful_module import increment_steps, init_states

    pcm = synth.gaussian(4, f"{tag}/pcm", n_frames * 1920, 0.1)
    with torch.no_grad():
        state = init_states(mimi, batch_size=1, sequence_length=1000)
        down_keys = [k for k in state if k.startswith("downsample") and "first" in state[k]]
        assert down_keys, "downsample conv state not found"
        lats = []
        for c0 in range(0, n_frames, chunk_frames):
            c1 = min(n_frames, c0 + chunk_frames)
            x = torch.from_numpy(pcm[c0 * 1920:c1 * 1920])[None, None]
            emb = mimi.encoder(x, model_state=state)
            (tr,) = mimi.encoder_transformer(emb, state)
            for k in down_keys:
                state[k]["first"][:] = True
            lats.append(mimi.downsample(tr, model_state=state))
            increment_steps(mimi, state, increment=tr.shape[-1])
        lat = torch.cat(lats, dim=-1)
        cond = torch.nn.functional.linear(lat.transpose(-1, -2), speaker_proj)
        # one-pass encode of the same PCM (tts_model.py:258-262), for the quirk's size
        one = mimi._to_framerate(mimi.encoder_transformer(mimi.encoder(torch.from_numpy(pcm)[None, None], None),
                                                          None)[0])
    return {"pcm": pcm, "latent": lat[0].numpy(), "conditioning": cond[0].numpy(),
            "latent_one_pass": one[0].numpy(), "meta": np.array([SEED, n_frames, chunk_frames], np.int64)}


def run_resample(torch, tag):
    """The Python reference's resampler, `convert_audio` (data/audio_utils.py:8-28, scipy
    resample_poly with the default Kaiser(5.0) FIR), on synthetic mono signals."""
    from pocket_tts.data.audio_utils import convert_audio

    out = {}
    for i, (sr, n) in enumerate(((48000, 12345), (44100, 8821), (16000, 4000), (22050, 5001), (8000, 1))):
        t = np.arange(n) / sr
        x = (0.5 * np.sin(2 * np.pi * 440.0 * t) + 0.3 * synth.gaussian(5 + i, f"{tag}/{sr}", n, 0.3)).astype(np.float32)
        y = convert_audio(torch.from_numpy(x)[None], sr, 24000, 1)[0].numpy()
        out[f"x_{sr}"] = x
        out[f"y_{sr}"] = np.ascontiguousarray(y, np.float32)
    # The reference's own real-data pair (its test_input_parity, parity_tests.rs:379-433):
    # assets/ref.wav (48 kHz s16 mono) and assets/ref_mimi_input.safetensors (its convert_audio
    # output, zero-padded to whole frames). Output sample m reads input samples <= 2m + 20, so the
    # head below is exact: the first 0.5 s of output and the input samples it depends on.
    import wave

    with wave.open(str(REF.parent / "assets" / "ref.wav"), "rb") as w:
        raw = np.frombuffer(w.readframes(w.getnframes()), np.int16)
    from safetensors.numpy import load_file

    mimi_input = load_file(str(REF.parent / "assets" / "ref_mimi_input.safetensors"))["mimi_input"].reshape(-1)
    out["refwav_head_i16"] = np.ascontiguousarray(raw[:24064])
    out["ref_mimi_input_head"] = np.ascontiguousarray(mimi_input[:12000], np.float32)
    out["ref_lengths"] = np.array([raw.size, mimi_input.size], np.int64)
    return out


def main():
    torch = _import_reference()
    torch.set_num_threads(8)
    from safetensors.numpy import save_file

    flm, mimi, speaker_proj = build_models(torch)
    if len(sys.argv) > 1 and sys.argv[1] == "refdata":  # the reference's own real-data fixtures, as data
        import shutil
        import wave

        from safetensors.numpy import load_file

        with wave.open(str(REF.parent / "assets" / "ref.wav"), "rb") as w:
            assert (w.getnchannels(), w.getsampwidth(), w.getframerate()) == (1, 2, 48000)
            raw = np.frombuffer(w.readframes(w.getnframes()), np.int16)
        mi = load_file(str(REF.parent / "assets" / "ref_mimi_input.safetensors"))["mimi_input"].reshape(-1)
        save_file({"refwav_i16": np.ascontiguousarray(raw), "ref_mimi_input": np.ascontiguousarray(mi, np.float32)},
                  str(HERE / "ref_voice.safetensors"))
        # real-weight intermediates of the reference's test_decoder_parity / voice conditioning
        # (meaningful only with the gated checkpoint; the weights-gated GPU tests use them)
        for f in ("ref_decoder_intermediates.safetensors", "ref_voice_conditioning.safetensors"):
            shutil.copyfile(REF.parent / "assets" / f, HERE / f)
        print("reference data fixtures written to", HERE)
        return
    if len(sys.argv) > 1 and sys.argv[1] == "names":  # the checkpoint's tensor names and shapes
        import json

        sd = {**{"flow_lm." + k: list(v.shape) for k, v in flm.state_dict().items()},
              **{"mimi." + k: list(v.shape) for k, v in mimi.state_dict().items()},
              "flow_lm.speaker_proj_weight": [1024, 512]}
        with open(HERE / "checkpoint_names.json", "w") as f:
            json.dump(sd, f, indent=0, sort_keys=True)
        print(len(sd), "names written to", HERE / "checkpoint_names.json")
        return
    if len(sys.argv) > 1 and sys.argv[1] == "long":  # the bench shape (BASELINE configs[2]) at B = 1
        # 125-frame "10 s" voice prompt, 40 text tokens, 100 free-running frames at temp 0: the
        # FlowLM context grows 165 -> 265 (past 256 keys) and the Mimi decoder's 250-key window
        # slides over 1600 positions (attention.rs:167-264, sdpa.rs:128-171)
        fx = run_e2e(torch, flm, mimi, F=125, S=40, N=100, lsd_steps=1, tag="e2e_long")
        del fx["tout"]
        save_file({k: np.ascontiguousarray(v) for k, v in fx.items()}, str(HERE / "e2e_long.safetensors"))
        print("long fixture written to", HERE)
        return
    if len(sys.argv) > 1 and sys.argv[1] == "hello":  # BASELINE configs[0] on synthetic weights
        # "Hello, world!" through the Rust segment driver (tts_model.rs:935-1071): prepare_text_prompt
        # gives "        Hello, world!" (2 words < 5: 8 spaces prepended), whose ids under the
        # reference's tokenizer.json are text_ids.json reference.native_ids[1] (tokenizers library,
        # gen_text_golden.py); temp 0, eos_threshold -4.0 (the CLI default), max_gen_len (2 + 2) * 13,
        # frames_after_eos 5 (estimate_frames_after_eos: <= 4 words). Voice "alba" is unavailable
        # offline: a synthetic 125-frame prompt stands in.
        import json

        tj = json.load(open(HERE / "text_ids.json"))
        assert tj["texts"][1] == "        Hello, world!"
        ids = tj["reference"]["native_ids"][1]
        # also at a threshold above every logit of the run: the segment then ends at max_gen_len
        for thr, name in ((-4.0, "hello_world"), (0.25, "hello_world_maxlen")):
            fx = run_e2e(torch, flm, mimi, F=125, S=len(ids), N=(2 + 2) * 13, lsd_steps=1, tag="hello",
                         ids=ids, eos_threshold=thr, frames_after_eos=5)
            del fx["tout"]
            save_file({k: np.ascontiguousarray(v) for k, v in fx.items()}, str(HERE / f"{name}.safetensors"))
            print(name, "stop", fx["stop"], "eos logits", fx["eos_logit"].min(), fx["eos_logit"].max())
        return
    if len(sys.argv) > 1 and sys.argv[1] == "voice":  # only the voice-cloning front-end fixtures
        fx = run_encoder_chunked(torch, mimi, speaker_proj, n_frames=5, chunk_frames=2, tag="encc5")
        save_file({k: np.ascontiguousarray(v) for k, v in fx.items()}, str(HERE / "encoder_chunked_5f.safetensors"))
        save_file(run_resample(torch, "resample"), str(HERE / "resample.safetensors"))
        print("voice fixtures written to", HERE)
        return
    fx = run_e2e(torch, flm, mimi, F=20, S=10, N=12, lsd_steps=1, tag="e2e_lsd1")
    save_file({k: np.ascontiguousarray(v) for k, v in fx.items()}, str(HERE / "e2e_lsd1.safetensors"))
    fx = run_e2e(torch, flm, mimi, F=8, S=6, N=4, lsd_steps=2, tag="e2e_lsd2")
    save_file({k: np.ascontiguousarray(v) for k, v in fx.items()}, str(HERE / "e2e_lsd2.safetensors"))
    fx = run_encoder(torch, mimi, speaker_proj, n_frames=4, tag="enc4")
    save_file({k: np.ascontiguousarray(v) for k, v in fx.items()}, str(HERE / "encoder_4f.safetensors"))
    # a few individual weights, to pin the PRNG restatement in C against numpy
    names = ["flow_lm.transformer.layers.0.self_attn.in_proj.weight", "flow_lm.bos_emb",
             "mimi.decoder.model.2.convtr.weight", "flow_lm.transformer.layers.3.norm2.bias",
             "mimi.decoder_transformer.transformer.layers.1.layer_scale_2.scale"]
    sd = {**{"flow_lm." + k: v for k, v in flm.state_dict().items()},
          **{"mimi." + k: v for k, v in mimi.state_dict().items()}}
    save_file({n: np.ascontiguousarray(sd[n].numpy().reshape(-1)[:4096]) for n in names},
              str(HERE / "synth_weights_head.safetensors"))
    print("fixtures written to", HERE)


if __name__ == "__main__":
    main()
