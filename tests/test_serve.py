"""Serving front end on CPU: continuous-batching scheduler logic and the HTTP
routes, driven by a stand-in engine with the ptts_slots_open / ptts_step contract (sequential and
pipelined frame delivery). The real-engine run of the same scheduler is a GPU parity test."""

import io
import struct
import wave
from types import SimpleNamespace

import numpy as np
import pytest

from pocket_tts_amd import GenerationParams
from pocket_tts_amd.serve import BatchScheduler, MultiGpuScheduler, TTSService, create_app, pcm_i16_le_bytes, wav_bytes


class FakeEngine:
    """Row r of step k of utterance u yields a frame filled with u*1000 + k; the last frame is
    flagged at max_frames. pipeline=True delivers each frame one call later (ptts_engine_config)."""

    def __init__(self, max_slots=4, pipeline=False):
        self.max_slots, self.max_ctx, self.pipeline = max_slots, 10_000, pipeline
        self.rows = {}
        self.pending = None
        self.calls = 0
        self.admissions = []

    def open_many(self, slots, voices, ids_list, params_list):
        self.admissions.append(list(slots))
        for s, ids, p in zip(slots, ids_list, params_list):
            self.rows[s] = {"u": int(ids[0]), "k": 0, "n": p.max_frames}
            if self.pending is not None:  # admission discards the slot's undrained frame
                self.pending["valid"][s] = False

    def _compute(self, n):
        out = {"pcm": np.zeros((n, 1920), np.float32), "valid": np.zeros(n, bool), "last": np.zeros(n, bool)}
        for s, st in list(self.rows.items()):
            if s >= n:
                continue
            out["pcm"][s] = st["u"] * 1000 + st["k"]
            out["valid"][s] = True
            st["k"] += 1
            out["last"][s] = st["k"] == st["n"]
            if out["last"][s]:
                del self.rows[s]
        return out

    def step(self, n):
        self.calls += 1
        cur = self._compute(n)
        if not self.pipeline:
            return SimpleNamespace(**cur)
        prev, self.pending = self.pending, cur
        if prev is None:
            return SimpleNamespace(pcm=np.zeros((n, 1920), np.float32), valid=np.zeros(n, bool),
                                   last=np.zeros(n, bool))
        m = min(n, prev["valid"].size)
        r = SimpleNamespace(pcm=np.zeros((n, 1920), np.float32), valid=np.zeros(n, bool), last=np.zeros(n, bool))
        r.pcm[:m], r.valid[:m], r.last[:m] = prev["pcm"][:m], prev["valid"][:m], prev["last"][:m]
        return r

    # split form of step() (ptts_step_async / ptts_sync / ptts_fetch[_prev]), used by the scheduler
    def step_async(self, n):
        self._issued = getattr(self, "_issued", [])[-1:] + [(self.step(n), n)]

    def sync(self):
        pass

    def fetch(self, n, calls_back=0):
        r, m = self._issued[-1 - calls_back]
        assert m == n
        return r


VOICE = SimpleNamespace(n_frames=10)


def params(n):
    return GenerationParams(temp=0.0, eos_threshold=float("inf"), max_frames=n, seed=1)


@pytest.mark.parametrize("pipeline", [False, True])
def test_scheduler_continuous_batching(pipeline):
    eng = FakeEngine(max_slots=4, pipeline=pipeline)
    sch = BatchScheduler(eng)
    try:
        lens = [5, 1, 3, 7, 2, 4, 6, 3, 1, 8]  # 10 requests through 4 slots
        reqs = [sch.submit([u + 1, 7, 7], VOICE, params(n)) for u, n in enumerate(lens)]
        for u, (req, n) in enumerate(zip(reqs, lens)):
            frames = list(req.stream(timeout=10))
            assert len(frames) == n
            assert [int(f[0]) for f in frames] == [(u + 1) * 1000 + k for k in range(n)]
        assert all(len(a) <= 4 for a in eng.admissions)
        assert sum(len(a) for a in eng.admissions) == len(lens)
        # continuous batching: far fewer engine calls than running the requests one by one
        assert eng.calls < sum(lens) - 10
    finally:
        sch.close()


class PreviewFakeEngine(FakeEngine):
    """Pipelined stand-in with first-frame previews (ptts_preview_enable / _fetch): a row's frame 0
    is also published as a preview `delay` fetch_previews() calls after the step that computed it
    (delay large: the regular frame 0 arrives first and the preview must be dropped)."""

    def __init__(self, max_slots=4, delay=0):
        super().__init__(max_slots=max_slots, pipeline=True)
        self.delay, self.pv, self.pv_rows = delay, [], 0

    def enable_preview(self, n):
        self.pv_rows = n

    def open_many(self, slots, *a):  # a re-admitted slot's unfetched preview is dropped (pv_forget)
        self.pv = [e for e in self.pv if e[1] not in slots]
        super().open_many(slots, *a)

    def _compute(self, n):
        starting = [s for s, st in self.rows.items() if s < n and st["k"] == 0][: self.pv_rows]
        out = super()._compute(n)
        for s in starting:
            self.pv.append([self.delay, s, out["pcm"][s].copy()])
        return out

    def fetch_ready(self, calls_back=0):
        return True

    def fetch_previews(self, wait=False):
        ready = [(s, p) for d, s, p in self.pv if d <= 0]
        self.pv = [[d - 1, s, p] for d, s, p in self.pv if d > 0]
        return ready


@pytest.mark.parametrize("delay", [0, 50])
def test_scheduler_first_frame_previews(delay):
    """The preview is delivered as frame 0 and the regular frame 0 dropped (delay 0), or the regular
    frame 0 comes first and the late preview is dropped (delay 50): every stream gets each frame
    exactly once, in order."""
    eng = PreviewFakeEngine(max_slots=3, delay=delay)
    sch = BatchScheduler(eng, preview_rows=2)
    try:
        lens = [4, 1, 3, 6, 2, 5, 1]
        reqs = [sch.submit([u + 1, 7], VOICE, params(n)) for u, n in enumerate(lens)]
        for u, (req, n) in enumerate(zip(reqs, lens)):
            assert [int(f[0]) for f in req.stream(timeout=10)] == [(u + 1) * 1000 + k for k in range(n)]
        assert (sch.previews > 0) == (delay == 0)
        assert sch.row_frames == sum(lens)
    finally:
        sch.close()


def test_multi_gpu_scheduler_spreads_requests():
    scheds = [BatchScheduler(FakeEngine(max_slots=2)) for _ in range(3)]
    multi = MultiGpuScheduler(scheds)
    try:
        reqs = [multi.submit([u + 1], [VOICE] * 3, params(4)) for u in range(9)]
        for u, r in enumerate(reqs):
            assert [int(f[0]) for f in r.stream(timeout=10)] == [(u + 1) * 1000 + k for k in range(4)]
        assert all(s.engine.calls > 0 for s in scheds)
    finally:
        multi.close()


def test_wire_formats_match_reference_rules():
    x = np.array([0.0, 0.5, -0.5, 1.0, -1.0, 2.0, -3.0, 0.99999, -0.00001], np.float32)
    got = np.frombuffer(pcm_i16_le_bytes(x), "<i2")
    # audio.rs:139-140: clamp to [-1, 1], * 32767, truncate toward zero
    assert got.tolist() == [0, 16383, -16383, 32767, -32767, 32767, -32767, 32766, 0]
    w = wave.open(io.BytesIO(wav_bytes(x)), "rb")
    assert (w.getnchannels(), w.getsampwidth(), w.getframerate(), w.getnframes()) == (1, 2, 24000, x.size)
    assert w.readframes(x.size) == pcm_i16_le_bytes(x)


def test_http_routes():
    from fastapi.testclient import TestClient

    sch = BatchScheduler(FakeEngine(max_slots=2, pipeline=True))
    svc = TTSService(sch, {"alba": VOICE}, default_voice="alba", tokenizer=lambda s: [5] * len(s.split()))
    try:
        c = TestClient(create_app(svc))
        assert c.get("/health").json()["status"] == "healthy"
        r = c.post("/generate", json={"token_ids": [3, 1, 2, 2], "words": 2})  # max_gen_len (2+2)*13 = 52 frames
        assert r.status_code == 200 and r.headers["content-type"] == "audio/wav"
        w = wave.open(io.BytesIO(r.content), "rb")
        assert w.getnframes() == 52 * 1920
        r = c.post("/stream", json={"text": "Hello world", "voice": "alba"})
        assert r.status_code == 200 and len(r.content) % (1920 * 2) == 0 and len(r.content) > 0
        r = c.post("/v1/audio/speech", json={"model": "pocket-tts", "input": "Hi there friend.",
                                             "response_format": "pcm"})
        assert r.status_code == 200 and len(r.content) % 3840 == 0
        assert c.post("/generate", json={"token_ids": [1], "words": 1, "voice": "nope"}).status_code == 400
        assert c.post("/generate", json={"token_ids": [1], "words": 1, "lsd_steps": 4}).status_code == 400
        assert c.post("/generate", json={}).status_code == 400
    finally:
        sch.close()


def test_stream_batches_coalesces_backlog():
    """A client behind the engine receives every frame already produced as one chunk, in order."""
    from pocket_tts_amd.serve import Request

    req = Request(np.zeros(3, np.int32), VOICE, params(5))
    for k in range(3):
        req.out.put(np.full(1920, k, np.float32))
    it = req.stream_batches(timeout=1)
    first = next(it)
    assert first.shape == (3 * 1920,) and [int(first[i * 1920]) for i in range(3)] == [0, 1, 2]
    req.out.put(np.full(1920, 3, np.float32))
    req.out.put(None)
    rest = list(it)
    assert len(rest) == 1 and rest[0].shape == (1920,) and int(rest[0][0]) == 3



def test_multiprocess_server_one_worker_per_gpu(tmp_path):
    """`serve --gpus 2` (CPU self-test: stand-in engines, gloo): the parent launches 2 worker
    processes as torch.distributed ranks (a child process, never exec); rank 0's weight blob
    reaches rank 1 through the load-time broadcast; both workers serve the SAME port
    (SO_REUSEPORT, the kernel spreads connections, no proxy hop) and answer /generate with their
    own engine's frames."""
    import os
    import signal
    import socket
    import subprocess
    import sys
    import time

    import httpx

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    np.save(tmp_path / "v.npy", np.zeros((4, 1024), np.float32))
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    env = dict(os.environ, PYTHONPATH=os.path.join(root, "pocket-tts_amd"))
    p = subprocess.Popen([sys.executable, "-m", "pocket_tts_amd.serve", "--gpus", "2", "--stand-in-engine",
                          "--port", str(port), "--slots", "4", "--voice", f"v={tmp_path / 'v.npy'}"],
                         env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, start_new_session=True)
    try:
        base = f"http://127.0.0.1:{port}"
        deadline = time.time() + 120
        while True:
            try:
                if httpx.get(base + "/health", timeout=2).status_code == 200:
                    break
            except httpx.HTTPError:
                pass
            assert p.poll() is None and time.time() < deadline, p.stdout.read().decode()[-3000:]
            time.sleep(0.5)
        seen, sums = set(), set()
        for i in range(40):
            with httpx.Client(timeout=30) as c:  # a fresh connection each time
                h = c.get(base + "/health").json()["worker"]
                seen.add(h["rank"])
                sums.add(h["weights_checksum"])
                r = c.post(base + "/generate", json={"token_ids": [7, 1, 2], "words": 1, "eos_threshold": 1e9})
                assert r.status_code == 200 and r.headers["x-ptts-rank"] in ("0", "1")
                pcm = np.frombuffer(r.content[44:], "<i2")
                assert pcm.size == (1 + 2) * 13 * 1920  # max_gen_len for 3 ids, stand-in frames
            if seen == {0, 1} and i >= 8:
                break
        assert seen == {0, 1}, seen
        assert sums == {float(sum(range(1024)))}  # rank 1 holds rank 0's broadcast blob
    finally:
        os.killpg(p.pid, signal.SIGTERM)
        try:
            p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()


def test_token_ids_need_a_word_count():
    """Token ids carry no word count, so the reference's max_gen_len rule ((words + 2) * 13,
    tts_model.rs:968) needs the client's `words` (or an explicit max_frames); neither -> 400."""
    from fastapi.testclient import TestClient

    eng = FakeEngine(max_slots=2)
    sch = BatchScheduler(eng)
    try:
        c = TestClient(create_app(TTSService(sch, {"v": VOICE}, default_voice="v")))
        assert c.post("/generate", json={"token_ids": [3, 1]}).status_code == 400
        r = c.post("/generate", json={"token_ids": [3, 1], "max_frames": 5})
        assert r.status_code == 200 and len(r.content) == 44 + 5 * 1920 * 2
        r = c.post("/generate", json={"token_ids": [3, 1], "words": 6})
        assert r.status_code == 200 and len(r.content) == 44 + (6 + 2) * 13 * 1920 * 2
    finally:
        sch.close()


def _start_server(tmp_path, gpus, slots, extra=()):
    import os
    import socket
    import subprocess
    import sys
    import time

    import httpx

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    np.save(tmp_path / "v.npy", np.zeros((4, 1024), np.float32))
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    env = dict(os.environ, PYTHONPATH=os.path.join(root, "pocket-tts_amd"), OMP_NUM_THREADS="1")
    p = subprocess.Popen([sys.executable, "-m", "pocket_tts_amd.serve", "--gpus", str(gpus), "--stand-in-engine",
                          "--port", str(port), "--slots", str(slots), "--voice", f"v={tmp_path / 'v.npy'}", *extra],
                         env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, start_new_session=True)
    base = f"http://127.0.0.1:{port}"
    deadline = time.time() + 240
    ranks = set()
    while len(ranks) < gpus:  # every worker up (fresh connections land on different workers)
        try:
            ranks.add(httpx.get(base + "/health", timeout=2).json()["worker"]["rank"])
        except (httpx.HTTPError, KeyError):
            time.sleep(0.5)
        assert p.poll() is None and time.time() < deadline, p.stdout.read().decode()[-3000:]
    return p, base


def _stop_server(p):
    import os
    import signal
    import subprocess

    os.killpg(p.pid, signal.SIGTERM)
    try:
        p.wait(timeout=30)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        p.wait()


@pytest.mark.timeout(600)
def test_configs3_256_streams_over_8_workers(tmp_path):
    """BASELINE configs[3] readiness on the CPU: `serve --gpus 8` (8 worker processes, stand-in
    engines paced at 1 ms per step, 32 slots each, gloo) under 256 concurrent /stream clients, two
    bursts. Every stream completes with exactly its frames on the wire (audio.rs:110-185 rule:
    the stand-in's samples are exact 16-bit codes), and the load spreads: the SO_REUSEPORT hash is
    blind to load, so a worker with no free slot sends the request (307) to the least-loaded peer
    (LoadBoard); no worker serves less than half its 32-stream share. Replaces the reference's
    one-mutex server (pocket-tts-cli/src/server/handlers.rs:215-306, state.rs:66-69)."""
    import asyncio
    import collections

    import httpx

    from pocket_tts_amd.serve import stand_in_sample

    n_frames, n_streams = 40, 256
    p, base = _start_server(tmp_path, 8, 32, ("--stand-in-step-ms", "1"))
    try:
        async def one(client, u):
            body = {"token_ids": [u, 5, 6], "max_frames": n_frames, "eos_threshold": 1e9}
            chunks = []
            async with client.stream("POST", base + "/stream", json=body) as r:
                assert r.status_code == 200
                rank = int(r.headers["x-ptts-rank"])
                redirected = bool(r.history)
                async for c in r.aiter_bytes():
                    chunks.append(c)
            pcm = np.frombuffer(b"".join(chunks), "<i2")
            assert pcm.size == n_frames * 1920, (u, pcm.size)
            want = np.repeat([int(round(stand_in_sample(u, k) * 32767 - 0.5)) for k in range(n_frames)], 1920)
            assert np.array_equal(pcm, want), u
            return rank, redirected

        async def burst(first):
            limits = httpx.Limits(max_connections=n_streams + 8, max_keepalive_connections=n_streams + 8)
            async with httpx.AsyncClient(timeout=120, limits=limits, follow_redirects=True) as client:
                return await asyncio.gather(*(one(client, first + i) for i in range(n_streams)))

        for b in range(2):
            res = asyncio.run(burst(1000 * b))
            per_rank = collections.Counter(r for r, _ in res)
            print(f"burst {b}: streams per worker {dict(sorted(per_rank.items()))}, "
                  f"redirected {sum(x for _, x in res)}")
            assert len(res) == n_streams and sorted(per_rank) == list(range(8)), per_rank
            assert min(per_rank.values()) >= 16, per_rank
    finally:
        _stop_server(p)


def test_load_board_never_redirects_to_a_dead_or_stale_worker(tmp_path):
    """a board entry left by a crashed worker (or an earlier server on the same port)
    must not draw 307s, even once its pid has been reused by another process. Entries carry the
    worker's pid and process start time; a worker resets its own entry when it maps the board and
    clears it on close."""
    import os
    import subprocess
    import sys

    from pocket_tts_amd.serve import LoadBoard

    path = str(tmp_path / "board.load")
    b0 = LoadBoard(port=1, world=3, rank=0, max_rows=4, path=path)
    b0.publish(4)  # rank 0 is full
    # rank 1: an entry of a process that has exited (free slots, a port)
    p = subprocess.Popen([sys.executable, "-c", "pass"])
    p.wait()
    b0.v[1] = (0, 5001, p.pid, 1)
    # rank 2: a stale entry with no pid at all (an earlier board layout / run)
    b0.v[2] = (0, 5002, 0, 0)
    assert b0.redirect_target(4) is None
    # a live pid whose start time differs from the entry's: the pid was reused, not the worker
    me = os.getpid()
    assert LoadBoard._start_time(me) > 0
    b0.v[1] = (0, 5001, me, LoadBoard._start_time(me) + 1)
    assert b0.redirect_target(4) is None
    # a live peer with a free slot is a target; re-mapping as rank 1 resets the stale entry first
    b1 = LoadBoard(port=1, world=3, rank=1, max_rows=4, path=path)
    assert tuple(b0.v[1]) == (0, 0, b1.v[1, 2], LoadBoard._start_time(me))
    b1.set_private_port(6001)
    assert b0.redirect_target(4) == 6001
    b1.close()
    assert b0.redirect_target(4) is None
    b0.close(unlink=True)
