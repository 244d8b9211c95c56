"""GPU: the HTTP server started the way the multi-GPU deployment starts it (SURVEY §8 f1,
BASELINE configs[3]): `serve --gpus 1 --torchrun` launches the worker as a torch.distributed rank
(torch.distributed.run as a CHILD process; the rank joins an RCCL process group, broadcasts the
packed weights and finalizes from them), then one /stream request (the reference's streaming
route, pocket-tts-cli/src/server/handlers.rs:215-310) is checked against the oracle: the chunked
16-bit PCM equals the oracle's frames converted by the same wire rule (audio.rs:110-185: clamp,
x 32767, truncate) to within one LSB."""

import os
import signal
import socket
import subprocess
import sys
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _i16(x):
    return (np.clip(np.asarray(x, np.float32), -1.0, 1.0) * np.float32(32767.0)).astype(np.int16)


def test_serve_torchrun_worker_stream_matches_oracle(tmp_path, oracle):
    import httpx

    rng = np.random.default_rng(23)
    prompt = (0.11 * rng.standard_normal((10, 1024))).astype(np.float32)
    np.save(tmp_path / "v.npy", prompt)
    ids = [(k * 97 + 13) % 4000 for k in range(12)]
    frames = 6
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    env = dict(os.environ, PYTHONPATH=os.path.join(ROOT, "pocket-tts_amd"))
    log = open(tmp_path / "server.log", "w+")
    p = subprocess.Popen([sys.executable, "-m", "pocket_tts_amd.serve", "--gpus", "1", "--torchrun", "--port",
                          str(port), "--slots", "4", "--max-ctx", "128", "--voice", f"v={tmp_path / 'v.npy'}"],
                         env=env, stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
    try:
        base = f"http://127.0.0.1:{port}"
        deadline = time.time() + 240
        while True:
            try:
                h = httpx.get(base + "/health", timeout=2)
                if h.status_code == 200:
                    break
            except httpx.HTTPError:
                pass
            if p.poll() is not None or time.time() > deadline:
                log.seek(0)
                pytest.fail("server did not come up:\n" + log.read()[-3000:])
            time.sleep(0.5)
        worker = h.json()["worker"]
        assert worker["world"] == 1 and worker["rank"] == 0 and worker["weights_checksum"] is not None
        body = {"token_ids": ids, "max_frames": frames, "temperature": 0.0, "eos_threshold": 1e9}
        with httpx.stream("POST", base + "/stream", json=body, timeout=120) as r:
            r.raise_for_status()
            data = b"".join(r.iter_bytes())
        got = np.frombuffer(data, "<i2")
        assert got.size == frames * 1920
        s = oracle.new_state(128)
        s.prefill(prompt)
        s.prefill_tokens(np.asarray(ids, np.int32))
        lat, want = None, []
        for _ in range(frames):
            o = s.step(lat)
            lat = o["latent"]
            want.append(_i16(o["pcm"]))
        d = np.abs(got.astype(np.int32) - np.concatenate(want).astype(np.int32))
        assert d.max() <= 1, d.max()
    finally:
        os.killpg(p.pid, signal.SIGTERM)
        try:
            p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait(timeout=30)
        log.close()
