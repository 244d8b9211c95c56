"""Batched serving front end: continuous batching of TTS requests over
the engine's slots, and the reference server's HTTP surface on top of it.

The reference server serializes every generation behind one mutex
(pocket-tts-cli/src/server/state.rs:69) and runs one utterance at a time per process. Here a
`BatchScheduler` owns one engine (one GPU) and a driver thread:

  1. requests wait in a queue; whenever slots are free, all waiting requests that fit are
     admitted in ONE batched admission (`ptts_slots_open`: shared text-prefill pass);
  2. every engine step advances all admitted rows together (`ptts_step`), and each row's
     1920-sample frame is handed to its request's stream as soon as it exists;
  3. a row's slot is recycled when its last frame (EOS tail or max_gen_len) has been delivered.

Works with both stepping modes of the engine (with `pipeline=True` a row's frames arrive one
step after they are computed). `MultiGpuScheduler` spreads requests over one scheduler per GPU
(replicas, no inter-GPU traffic: DESIGN.md §6) inside one process; `main(--gpus N)` instead runs
one worker process per GPU, each a whole server on one shared SO_REUSEPORT port (the weights
packed once and broadcast over RCCL at load time).

HTTP (`create_app`, FastAPI; routes of pocket-tts-cli/src/server/routes.rs:20-30):
  GET  /health             {"status": "healthy", "version": ...}
  POST /generate           JSON {text | token_ids, voice?, temperature?, eos_threshold?,
                           noise_clamp?, lsd_steps?} -> audio/wav (handlers.rs:128-213)
  POST /stream             same body -> chunked 16-bit PCM LE (handlers.rs:215-310): the first
                           frame as soon as it exists, later frames coalesced to at most one
                           chunk per 20 ms per stream
  POST /v1/audio/speech    OpenAI body {model, input, voice?, response_format?} -> wav / pcm
                           (handlers.rs:380-398)
Wire formats follow crates/pocket-tts/src/audio.rs:110-185 (clamp to [-1, 1], x 32767,
truncate to i16; 16-bit mono RIFF/WAVE).
"""

from __future__ import annotations

import os
import queue
import struct
import threading
import time
from collections import deque
from dataclasses import dataclass, field
from typing import Callable, Iterator, Sequence

import numpy as np

from ._lib import FRAME, SAMPLE_RATE
from .audio import pcm_i16_le_bytes, wav_bytes  # noqa: F401 (re-exported wire formats)
from .engine import GenerationParams, Voice
from .text import estimate_frames_after_eos, max_gen_len, prepare_text_prompt

VERSION = "0.1.0"


# wire formats (audio.rs:110-185) live in .audio: pcm_i16_le_bytes, wav_bytes


class FrameChannel:
    """One producer (the scheduler thread), one consumer: the queue.Queue calls a Request's
    consumers use (put / get / get_nowait / empty), without a lock and condition round trip per
    frame. A deque append is atomic under the GIL, so put() is one append and, only while a
    consumer is blocked in get(), one notify (the scheduler delivers 32 frames per ~0.6-ms step:
    a locked Queue.put per frame cost it a large share of the step)."""

    def __init__(self):
        self._d: deque = deque()
        self._cv = threading.Condition(threading.Lock())
        self._waiting = False

    def put(self, item):
        self._d.append(item)
        if self._waiting:  # the consumer set this before it checked the deque: it sees either
            with self._cv:  # the appended item or this notify
                self._cv.notify()

    def get_nowait(self):
        try:
            return self._d.popleft()
        except IndexError:
            raise queue.Empty from None

    def empty(self) -> bool:
        return not self._d

    def get(self, timeout: float | None = None):
        try:
            return self._d.popleft()
        except IndexError:
            pass
        deadline = None if timeout is None else time.monotonic() + timeout
        with self._cv:
            self._waiting = True
            try:
                while not self._d:
                    rem = None if deadline is None else deadline - time.monotonic()
                    if rem is not None and rem <= 0:
                        raise queue.Empty
                    self._cv.wait(rem)
                return self._d.popleft()
            finally:
                self._waiting = False


# ---------------------------------------------------------------------------------------------
@dataclass
class Request:
    ids: np.ndarray
    voice: Voice
    params: GenerationParams
    out: FrameChannel = field(default_factory=FrameChannel)  # np.ndarray frames, then None
    slot: int = -1
    frames: int = 0
    waker: Callable[[], None] | None = None  # set by an async consumer (HTTP /stream)
    times: dict = field(default_factory=dict)  # submit / admit / first / last (time.time())
    # first-frame preview: 1 = the preview was delivered as frame 0 and the regular frame 0 is still
    # to come (it is dropped), 2 = that frame came
    preview: int = 0
    start_step: int = 0  # the scheduler's step that starts the row (trace)

    def put(self, item):
        """Driver side: hand over a frame (np.ndarray), the end marker (None) or an error."""
        self.out.put(item)
        w = self.waker
        if w is not None:
            w()

    def stream(self, timeout: float | None = None) -> Iterator[np.ndarray]:
        """Frames [1920] float32 as they are produced; raises the driver's error if any."""
        while True:
            item = self.out.get(timeout=timeout)
            if item is None:
                return
            if isinstance(item, BaseException):
                raise item
            yield item

    def stream_batches(self, timeout: float | None = None) -> Iterator[np.ndarray]:
        """Like stream(), but each item is every frame available at that moment, concatenated
        (at least one): a client that falls behind the engine gets one HTTP chunk per backlog
        instead of one per frame, so per-chunk server overhead cannot throttle the stream."""
        done = False
        while not done:
            frames = [self.out.get(timeout=timeout)]
            while True:
                try:
                    frames.append(self.out.get_nowait())
                except queue.Empty:
                    break
            batch = []
            for item in frames:
                if item is None:
                    done = True
                    break
                if isinstance(item, BaseException):
                    raise item
                batch.append(item)
            if batch:
                yield batch[0] if len(batch) == 1 else np.concatenate(batch)

    def audio(self, timeout: float | None = None) -> np.ndarray:
        frames = list(self.stream(timeout))
        return np.concatenate(frames) if frames else np.zeros(0, np.float32)


class BatchScheduler:
    """Continuous batching over one engine's slots (one GPU).

    On a pipelined engine a new row's first frame would trail its first step by the pipeline's
    frame lag (three calls with frame-pair passes). With `preview_rows` > 0 the engine also decodes
    each new row's first frame on its own right after that step (ptts_preview_enable); the
    scheduler delivers that preview as the request's frame 0 and drops the regular frame 0 when it
    comes (the two agree within float rounding: the regular pass decodes it from the same fresh
    state), or, if the regular frame comes first, drops the preview."""

    def __init__(self, engine, max_rows: int | None = None, preview_rows: int = 8):
        self.engine = engine
        self.max_rows = min(max_rows or engine.max_slots, engine.max_slots)
        self.preview = bool(preview_rows) and getattr(engine, "pipeline", False) and hasattr(engine, "enable_preview")
        if self.preview:
            engine.enable_preview(preview_rows)
        self.previews = 0  # first frames delivered from a preview
        self.poll_s = 50e-6
        self.shallow = getattr(engine, "pipeline", False) and hasattr(engine, "front_done")
        self.waiting: deque[Request] = deque()
        self.active: dict[int, Request] = {}
        self.cv = threading.Condition()
        self.running = True
        self.steps = 0
        self.row_frames = 0  # frames delivered (valid rows summed over steps)
        self.trace = bool(os.environ.get("PTTS_SERVE_TRACE"))
        # called (under self.cv) with the new load whenever it changes: the multi-process server
        # publishes it on its LoadBoard for the overflow redirect
        self.on_load: Callable[[int], None] | None = None
        self.thread = threading.Thread(target=self._loop, name="ptts-scheduler", daemon=True)
        self.thread.start()

    # -- client side
    def submit(self, ids, voice: Voice, params: GenerationParams) -> Request:
        req = Request(np.asarray(ids, np.int32).reshape(-1), voice, params)
        req.times["submit"] = time.time()
        if voice.n_frames + req.ids.size + params.max_frames > self.engine.max_ctx:
            raise ValueError("voice + text + max_frames exceeds the engine's max_ctx")
        with self.cv:
            if not self.running:
                raise RuntimeError("scheduler stopped")
            self.waiting.append(req)
            if self.on_load is not None:
                self.on_load(len(self.active) + len(self.waiting))
            self.cv.notify()
        return req

    def load(self) -> int:
        with self.cv:
            return len(self.active) + len(self.waiting)

    def close(self):
        with self.cv:
            self.running = False
            self.cv.notify()
        self.thread.join()

    # -- driver thread
    def _take(self) -> list[Request]:
        """(under self.cv) waiting requests that fit the free slots, slots assigned and reserved"""
        free = [s for s in range(self.max_rows) if s not in self.active]
        batch = []
        while self.waiting and free:
            req = self.waiting.popleft()
            req.slot = free.pop(0)
            self.active[req.slot] = req
            batch.append(req)
        return batch

    def _admit(self, batch: list[Request]):
        """(outside self.cv: submit() runs on the HTTP event loop and must never wait for an
        admission's engine call) one batched admission of the taken requests"""
        self.engine.open_many([r.slot for r in batch], [r.voice for r in batch], [r.ids for r in batch],
                              [r.params for r in batch])
        now = time.time()
        # the rows start at the step issued admit_delay calls after the next one (ptts_frame_lag)
        delay = self.engine.frame_lag()[1] if hasattr(self.engine, "frame_lag") else 0
        for r in batch:
            r.times["admit"] = now
            r.start_step = self.steps + delay

    def _deliver_previews(self):
        if not self.preview:
            return
        for slot, pcm in self.engine.fetch_previews():
            req = self.active.get(slot)
            if req is None or req.frames or req.preview:  # the regular frame 0 came first
                continue
            req.preview = 1
            req.frames = 1
            self.row_frames += 1
            self.previews += 1
            req.times["first"] = time.time()
            req.put(pcm)

    def _deliver(self, res, rows) -> list[int]:
        done = []
        for slot, req in list(self.active.items()):
            if slot < rows and res.valid[slot]:
                if req.preview == 1:  # frame 0, already delivered from the preview
                    req.preview = 2
                else:
                    req.frames += 1
                    self.row_frames += 1
                    if req.frames == 1:
                        req.times["first"] = time.time()
                    req.put(res.pcm[slot])  # a view: fetch() returns fresh arrays every step
                if res.last[slot]:
                    req.times["last"] = time.time()
                    if self.trace:
                        t = req.times
                        t0 = t.get("route", t["submit"])
                        ts = t.get("start", t["submit"])
                        print(f"ptts-serve slot {slot} route_to_submit_ms {1e3 * (t['submit'] - t0):.1f} "
                              f"start_ms {1e3 * (ts - t['submit']):.2f} "
                              f"first_after_start_ms {1e3 * (t['first'] - ts):.2f} "
                              f"first_to_chunk0_ms {1e3 * (t.get('chunk0', t['first']) - t['first']):.1f} "
                              f"frames {req.frames} admit_wait_ms "
                              f"{1e3 * (t['admit'] - t['submit']):.1f} first_ms {1e3 * (t['first'] - t['submit']):.1f} "
                              f"last_ms {1e3 * (t['last'] - t['submit']):.1f} steps {self.steps}", flush=True)
                    req.put(None)
                    done.append(slot)
        return done

    def _loop(self):
        # One call in flight: call k+1 is issued (step_async) before the frames of call k are
        # fetched and handed out, so the GPU always has the next step queued while this thread
        # waits for the GIL (the HTTP event loop shares it) and delivers frames. A finished row is
        # released when its last frame is delivered (later calls compute it as inactive:
        # frame_valid = 0).
        issued: deque[int] = deque()  # rows of the calls issued and not fetched yet (<= 2)
        try:
            while True:
                with self.cv:
                    while self.running and not self.waiting and not self.active and not issued:
                        self.cv.wait()
                    if not self.running:
                        break
                    batch = self._take()
                    rows = max(self.active) + 1 if self.active else 0
                # A pipelined engine lets the host run calls ahead of the GPU (the fetch below waits
                # for a frame several calls old), and an admission queues behind every FlowLM step
                # already issued: keep one step queued behind the running one, no more, so a new
                # row's prefill and first step wait for one step at most (first-chunk latency; the
                # GPU still always has the next step queued)
                if self.shallow and issued:
                    self.engine.front_done(1, wait=True)
                if batch:
                    self._admit(batch)
                if rows:
                    self.engine.step_async(rows)
                    issued.append(rows)
                    if self.trace:
                        now = time.time()
                        for r in self.active.values():
                            if r.start_step == self.steps:
                                r.times["start"] = now
                    self.steps += 1
                self._deliver_previews()
                if len(issued) == 2 or (issued and not rows):
                    cb = len(issued) - 1
                    # while a stream waits for its first frame, poll the call's frame and the
                    # previews (~50 us apart) instead of blocking in fetch(): a preview completes
                    # while the call's back pass still runs, and is handed out as soon as it does
                    if self.preview and any(r.frames == 0 for r in self.active.values()):
                        while not self.engine.fetch_ready(cb):
                            self._deliver_previews()
                            time.sleep(self.poll_s)
                    res = self.engine.fetch(issued[0], calls_back=cb)
                    self._deliver_previews()  # those that completed while fetch() waited: ahead of it
                    done = self._deliver(res, issued.popleft())
                    if done:
                        with self.cv:
                            for slot in done:
                                del self.active[slot]
                            if self.on_load is not None:
                                self.on_load(len(self.active) + len(self.waiting))
        except BaseException as e:  # deliver the failure to every waiting client
            with self.cv:
                self.running = False
                for req in list(self.active.values()) + list(self.waiting):
                    req.put(e)
                    req.put(None)
                self.active.clear()
                self.waiting.clear()
        finally:
            with self.cv:
                for req in list(self.active.values()) + list(self.waiting):
                    req.put(None)


class MultiGpuScheduler:
    """Replicas: one BatchScheduler per GPU engine; a request goes to the least loaded one."""

    def __init__(self, schedulers: Sequence[BatchScheduler]):
        self.schedulers = list(schedulers)

    def submit(self, ids, voices: Sequence[Voice], params: GenerationParams) -> Request:
        i = min(range(len(self.schedulers)), key=lambda k: self.schedulers[k].load())
        return self.schedulers[i].submit(ids, voices[i], params)

    def close(self):
        for s in self.schedulers:
            s.close()


class LoadBoard:
    """Least-loaded dispatch for the multi-process server (BASELINE configs[3]: 256 streams over 8
    GPUs). The kernel spreads connections over the workers of the shared SO_REUSEPORT port by a hash,
    blind to load, and a keep-alive connection stays on its worker; so each worker publishes its
    load (requests active + waiting) and the port of a private listener in one small file under
    /dev/shm that every worker of the server maps, and a worker with no free slot answers a request
    on the shared port with 307 (method and body kept) to the private port of the least-loaded peer
    that has one. Requests on a private port are always served (a request is redirected at most
    once). One int64 quadruple per rank: (load, private port, pid, process start time). Each worker
    resets its own entry when it maps the board, and a peer is a target only while a process with
    that pid AND that start time (/proc/<pid>/stat field 22) exists, so an entry left by a crashed
    worker, or by an earlier server on the same port, is not redirected to even after the pid has
    been reused by another process."""

    FIELDS = 4

    def __init__(self, port: int, world: int, rank: int, max_rows: int, path: str | None = None):
        import mmap

        self.world, self.rank, self.max_rows = world, rank, max_rows
        self.path = path or f"/dev/shm/ptts-serve-{port}-{world}.load"
        size = 8 * self.FIELDS * world
        fd = os.open(self.path, os.O_RDWR | os.O_CREAT, 0o600)
        try:
            if os.fstat(fd).st_size != size:
                os.ftruncate(fd, size)
            self._mm = mmap.mmap(fd, size)
        finally:
            os.close(fd)
        self.v = np.frombuffer(self._mm, np.int64).reshape(world, self.FIELDS)
        self.v[rank] = (0, 0, os.getpid(), self._start_time(os.getpid()))  # whatever an earlier run left
        self.private_port = 0

    def publish(self, load: int):
        self.v[self.rank, 0] = load

    def set_private_port(self, port: int):
        self.private_port = port
        self.v[self.rank, 1] = port

    @staticmethod
    def _start_time(pid: int) -> int:
        """The process's start time in clock ticks since boot (/proc/<pid>/stat field 22); -1 if
        there is no such process (0 where /proc is not available)."""
        try:
            with open(f"/proc/{int(pid)}/stat", "rb") as f:
                stat = f.read().decode(errors="replace")
        except FileNotFoundError:
            return -1
        except OSError:
            return 0
        # the command name (field 2) is parenthesised and may hold spaces: fields after its ')'
        return int(stat[stat.rindex(")") + 2:].split()[19])

    @classmethod
    def _alive(cls, pid: int, start: int = 0) -> bool:
        """True while the worker that published (pid, start) runs: a live process with that pid,
        owned by this user, started at that time (a reused pid has a later start time)."""
        if pid <= 0:
            return False
        try:
            os.kill(int(pid), 0)
        except ProcessLookupError:
            return False
        except PermissionError:  # exists, owned by another user: not one of this server's workers
            return False
        return start == 0 or cls._start_time(pid) == start

    def redirect_target(self, own_load: int) -> int | None:
        """The private port of the least-loaded live peer with a free slot, if this worker has none."""
        if own_load < self.max_rows:
            return None
        loads, ports, pids, starts = (self.v[:, i].copy() for i in range(self.FIELDS))
        best = None
        for r in range(self.world):
            if (r != self.rank and ports[r] > 0 and loads[r] < self.max_rows and (best is None or loads[r] < loads[best])
                    and self._alive(pids[r], starts[r])):
                best = r
        if best is None:
            return None
        self.v[best, 0] += 1  # claim the slot now: concurrent overflows spread instead of herding
        return int(ports[best])

    def close(self, unlink: bool = False):
        if self.v is not None:
            self.v[self.rank] = (0, 0, 0, 0)  # a closed worker is no target
        self.v = None
        self._mm.close()
        if unlink:
            try:
                os.unlink(self.path)
            except FileNotFoundError:
                pass


# ---------------------------------------------------------------------------------------------
def load_tokenizer(path: str) -> Callable[[str], list[int]]:
    """tokenizer.model (SentencePiece) or tokenizer.json; a .json file is read with the native
    Rust settings (text.rs:71-79: Metaspace prepend "always", no BOS), see text.py."""
    from .text import Tokenizer

    return Tokenizer.from_file(path, native=True)


class TTSService:
    """Request-level logic shared by the HTTP routes: text -> ids, voice lookup, params."""

    def __init__(self, scheduler, voices: dict[str, Voice | Sequence[Voice]], default_voice: str,
                 tokenizer: Callable[[str], Sequence[int]] | None = None, temp: float = 0.7,
                 eos_threshold: float = -4.0, noise_clamp: float | None = None, lsd_decode_steps: int = 1):
        self.scheduler = scheduler
        self.voices = voices
        self.default_voice = default_voice
        self.tokenizer = tokenizer
        self.temp, self.eos_threshold, self.noise_clamp = temp, eos_threshold, noise_clamp
        self.lsd_decode_steps = lsd_decode_steps
        self._seed = 0
        self._lock = threading.Lock()

    def request(self, text: str | None = None, token_ids=None, voice: str | None = None,
                temperature: float | None = None, eos_threshold: float | None = None,
                noise_clamp: float | None = None, lsd_steps: int | None = None, words: int | None = None,
                max_frames: int | None = None) -> Request:
        if lsd_steps is not None and lsd_steps != self.lsd_decode_steps:
            raise ValueError(f"lsd_steps is fixed at engine creation ({self.lsd_decode_steps})")
        if token_ids is not None:  # extension: ids carry no word count, the client states it
            ids = np.asarray(token_ids, np.int32).reshape(-1)
            if words is None and max_frames is None:
                raise ValueError("token_ids need `words` (word count of their text) or `max_frames`")
            mgl = max_frames or (words + 2) * 13
            fae = 3 if words is None else (5 if words <= 4 else 3)
        elif text is not None:
            if self.tokenizer is None:
                raise ValueError("no tokenizer configured: send token_ids")
            prepared = prepare_text_prompt(text)
            ids = np.asarray(self.tokenizer(prepared), np.int32)
            mgl, fae = max_frames or max_gen_len(prepared), estimate_frames_after_eos(text)
        else:
            raise ValueError("text or token_ids required")
        name = voice or self.default_voice
        if name not in self.voices:
            raise ValueError(f"unknown voice {name!r}")
        with self._lock:
            self._seed += 1
            seed = self._seed
        p = GenerationParams(temp=self.temp if temperature is None else temperature,
                             eos_threshold=self.eos_threshold if eos_threshold is None else eos_threshold,
                             noise_clamp=self.noise_clamp if noise_clamp is None else noise_clamp,
                             frames_after_eos=fae, max_frames=mgl, seed=seed)
        return self.scheduler.submit(ids, self.voices[name], p)  # MultiGpuScheduler: one voice per GPU


from pydantic import BaseModel  # noqa: E402  (request bodies; module level so FastAPI resolves them)
from starlette.requests import Request as StarletteRequest  # noqa: E402


class GenerateRequest(BaseModel):
    """handlers.rs:84-92 (+ token_ids when no tokenizer is configured)."""

    text: str | None = None
    token_ids: list[int] | None = None
    words: int | None = None  # with token_ids: word count of their text (max_gen_len rule)
    max_frames: int | None = None
    voice: str | None = None
    temperature: float | None = None
    lsd_steps: int | None = None
    eos_threshold: float | None = None
    noise_clamp: float | None = None


class OpenAIRequest(BaseModel):
    """handlers.rs:378-385."""

    model: str = "pocket-tts"
    input: str | None = None
    voice: str | None = None
    response_format: str | None = None
    token_ids: list[int] | None = None
    words: int | None = None


# /stream: at most one chunk per stream per 20 ms after the first (32 streams x 50 wakes/s keep the
# event loop, which shares the GIL with the scheduler thread, well below one core)
CHUNK_INTERVAL_S = 0.02


async def pcm_chunks(r: Request):
    """/stream body without a worker thread per stream. The driver's put() wakes this coroutine
    on the event loop (call_soon_threadsafe, at most one pending wake per stream); each wake
    sends every frame available at that moment as ONE chunk of 16-bit PCM, then the stream
    waits CHUNK_INTERVAL_S before the next. The first frame goes out as soon as it exists; later
    frames coalesce, so 32 streams of a GPU producing ~4000x real time cost at most 50 chunks/s
    each instead of one event-loop round trip per 80-ms frame (which throttled the whole server).
    """
    import asyncio

    loop = asyncio.get_running_loop()
    ev = asyncio.Event()
    armed = [False]

    def wake():
        if armed[0]:
            armed[0] = False
            loop.call_soon_threadsafe(ev.set)

    r.waker = wake
    while True:
        items = []
        while True:
            try:
                items.append(r.out.get_nowait())
            except queue.Empty:
                break
        batch, done = [], False
        for item in items:
            if item is None:
                done = True
                break
            if isinstance(item, BaseException):
                raise item
            batch.append(item)
        if batch:
            if "chunk0" not in r.times:
                r.times["chunk0"] = time.time()
            yield pcm_i16_le_bytes(batch[0] if len(batch) == 1 else np.concatenate(batch))
        if done:
            return
        if batch:
            await asyncio.sleep(CHUNK_INTERVAL_S)
        ev.clear()
        armed[0] = True
        if r.out.empty():
            await ev.wait()


def create_app(service: TTSService):
    from fastapi import FastAPI, HTTPException
    from fastapi.responses import JSONResponse, Response, StreamingResponse

    app = FastAPI(title="pocket-tts (MI355X engine)")

    def submit(**kw) -> Request:
        try:
            return service.request(**kw)
        except ValueError as e:
            raise HTTPException(status_code=400, detail=str(e)) from e

    worker = getattr(service, "worker", None) or {"rank": 0, "world": 1, "pid": os.getpid()}
    hdr = {"X-PTTS-Rank": str(worker["rank"])}
    board: LoadBoard | None = getattr(service, "board", None)
    shared_port = getattr(service, "shared_port", None)

    def overflow(request):
        """A 307 to the least-loaded peer's private port when this worker has no free slot and the
        request came in on the shared port (LoadBoard); None to serve it here."""
        if board is None or request.scope.get("server", (None, None))[1] != shared_port:
            return None
        from fastapi.responses import RedirectResponse

        port = board.redirect_target(service.scheduler.load())
        if port is None:
            return None
        return RedirectResponse(str(request.url.replace(port=port)), status_code=307, headers=hdr)

    @app.get("/health")
    def health():
        sch = getattr(service, "scheduler", None)
        stats = {"steps": sch.steps, "frames": sch.row_frames} if isinstance(sch, BatchScheduler) else {}
        return JSONResponse({"status": "healthy", "version": VERSION, "worker": worker, **stats}, headers=hdr)

    @app.post("/generate")
    def generate(req: GenerateRequest, request: StarletteRequest):
        redirect = overflow(request)
        if redirect is not None:
            return redirect
        r = submit(**req.model_dump())
        return Response(wav_bytes(r.audio()), media_type="audio/wav", headers=hdr)

    @app.post("/stream")
    async def stream(req: GenerateRequest, request: StarletteRequest):
        t_route = time.time()
        redirect = overflow(request)
        if redirect is not None:
            return redirect
        r = submit(**req.model_dump())
        r.times["route"] = t_route
        return StreamingResponse(pcm_chunks(r), media_type="audio/pcm",
                                 headers={**hdr, "X-PTTS-Route-Time": f"{t_route:.6f}"})

    @app.post("/v1/audio/speech")
    def openai_speech(req: OpenAIRequest, request: StarletteRequest):
        redirect = overflow(request)
        if redirect is not None:
            return redirect
        r = submit(text=req.input, token_ids=req.token_ids, voice=req.voice, words=req.words)
        audio = r.audio()
        if (req.response_format or "wav") == "pcm":
            return Response(pcm_i16_le_bytes(audio), media_type="audio/pcm", headers=hdr)
        return Response(wav_bytes(audio), media_type="audio/wav", headers=hdr)

    return app


def stand_in_sample(u: int, k: int) -> float:
    """The stand-in engine's sample value for utterance u (its first token id) at frame k: the
    16-bit wire value (audio.rs:110-185: x 32767, truncated) is exactly (u % 128) * 256 + k % 256."""
    return ((u % 128) * 256 + k % 256 + 0.5) / 32767.0


class StandInEngine:
    """--stand-in-engine only (CPU; launcher and routing self-test of the multi-process server): the
    engine surface the scheduler drives, computing nothing. Row frames of utterance u (its first
    token id) at step k hold stand_in_sample(u, k), delivered one call late as by a pipelined
    engine; step_s paces each step (sleep) like a GPU step."""

    def __init__(self, max_slots=32, max_ctx=1024, step_s=0.0, **_):
        self.max_slots, self.max_ctx, self.pipeline = max_slots, max_ctx, True
        self.step_s = step_s
        self.rows, self.pending = {}, None

    @staticmethod
    def weight_blob_bytes():
        return 4096

    def finalize(self):
        pass

    def voice_from_prompt(self, prompt):
        from types import SimpleNamespace

        return SimpleNamespace(n_frames=int(np.asarray(prompt).shape[0]))

    def open_many(self, slots, voices, ids_list, params_list):
        for s, ids, p in zip(slots, ids_list, params_list):
            self.rows[s] = [int(ids[0]) if len(ids) else 0, 0, p.max_frames]
            if self.pending is not None and s < self.pending[1].size:  # drop the slot's undrained frame
                self.pending[1][s] = False

    def step_async(self, n):
        if self.step_s:
            time.sleep(self.step_s)
        pcm, valid, last = np.zeros((n, FRAME), np.float32), np.zeros(n, bool), np.zeros(n, bool)
        for s, st in list(self.rows.items()):
            if s < n:
                pcm[s], valid[s] = stand_in_sample(st[0], st[1]), True
                st[1] += 1
                last[s] = st[1] == st[2]
                if last[s]:
                    del self.rows[s]
        prev, self.pending = self.pending, (pcm, valid, last)
        self.prev_out = getattr(self, "out", None)
        self.out = (np.zeros((n, FRAME), np.float32), np.zeros(n, bool), np.zeros(n, bool))
        if prev is not None:  # the previous call's frame, over this call's rows
            m = min(n, prev[1].size)
            for a, b in zip(self.out, prev):
                a[:m] = b[:m]

    def sync(self):
        pass

    def fetch(self, n, calls_back=0):
        from types import SimpleNamespace

        out = self.out if calls_back == 0 else self.prev_out
        return SimpleNamespace(pcm=out[0], valid=out[1], last=out[2])

    def close(self):
        pass


def _listen_socket(host: str, port: int, reuse_port: bool = True):
    """A listening TCP socket with SO_REUSEPORT: every per-GPU worker process binds the same port
    and the kernel spreads incoming connections over them (no proxy process in the data path)."""
    import socket

    # proto IPPROTO_TCP explicitly: asyncio sets TCP_NODELAY only on transports whose socket says
    # so (proto 0 left Nagle on: every chunk written behind the response headers waited for the
    # client's delayed ACK, ~20 ms on a stream's first chunk); the listener's NODELAY is inherited
    so = socket.socket(socket.AF_INET, socket.SOCK_STREAM, socket.IPPROTO_TCP)
    so.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
    so.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    if reuse_port:
        so.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEPORT, 1)
    so.bind((host, port))
    so.listen(1024)
    return so


def _worker_engine(args, Engine):
    """This process's engine. Under torch.distributed (one rank per GPU): rank 0 packs the weights
    (checkpoint or synthetic) into its engine-owned blob, ONE broadcast over RCCL (xGMI) copies it
    to every rank at load time, the other ranks finalize from it (no per-step
    collective). Returns (engine, rank, world, blob checksum)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    kw = dict(max_slots=args.slots, max_ctx=args.max_ctx, weights_path=args.weights, pipeline=True,
              back_frames=args.back_frames)
    if Engine is StandInEngine:
        kw["step_s"] = args.stand_in_step_ms / 1000.0
    if "WORLD_SIZE" not in os.environ:  # a plain single-GPU server
        return Engine(device=local, **kw), 0, 1, None
    import torch
    import torch.distributed as dist

    stand_in = Engine is StandInEngine
    if not stand_in:
        torch.cuda.set_device(local)
    dist.init_process_group("gloo" if stand_in else "nccl")
    dev = "cpu" if stand_in else f"cuda:{local}"
    blob = torch.empty(Engine.weight_blob_bytes() // 4, dtype=torch.float32, device=dev)
    if stand_in and rank == 0:
        blob.copy_(torch.arange(blob.numel(), dtype=torch.float32))
    eng = Engine(device=local, weight_blob=blob.data_ptr(), defer_weights=rank != 0, **kw)
    if not stand_in:
        torch.cuda.synchronize()
    dist.broadcast(blob, src=0)
    if not stand_in:
        torch.cuda.synchronize()
    if rank != 0:
        eng.finalize()
    checksum = float(blob[:1024].double().sum().item())
    dist.barrier()
    return eng, rank, world, checksum


def main(argv=None):
    """python -m pocket_tts_amd.serve --voice NAME=prompt.npy [--voice ...] [--tokenizer t.json]
    [--gpus N] [--slots 32] [--port 8000]

    --gpus N > 1: one worker PROCESS per GPU (launched as N ranks of torch.distributed.run, a
    child process; this parent never touches the GPU), each with its own engine, scheduler and
    HTTP server on the same SO_REUSEPORT port: no shared GIL, no proxy hop; the weights are packed
    once and broadcast over RCCL at load time."""
    import argparse

    # before any HIP initialization (a torchrun worker's RCCL setup comes before the engine library
    # loads, which sets the same default): graph kernel nodes instead of captured packets (capi.cpp)
    os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")

    ap = argparse.ArgumentParser()
    ap.add_argument("--voice", action="append", default=[], help="NAME=path (.npy prompt [F,1024] or .wav)")
    ap.add_argument("--tokenizer", default=None)
    ap.add_argument("--weights", default=None)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--torchrun", action="store_true",
                    help="launch the worker(s) as torch.distributed ranks even for --gpus 1 (the N-GPU path)")
    ap.add_argument("--slots", type=int, default=32)
    ap.add_argument("--max-ctx", type=int, default=1024)
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8000)
    ap.add_argument("--back-frames", type=int, default=2, choices=(1, 2, 4, 8),
                    help="frames per Mimi decode pass (ptts_engine_config.back_frames): 2, the throughput "
                         "configuration bench.py measures (two more calls of frame lag, ~1.2 ms at B = 32)")
    ap.add_argument("--preview-rows", type=int, default=8,
                    help="first-frame previews: rows per call whose first frame is decoded at once (0: off)")
    ap.add_argument("--stand-in-engine", action="store_true",
                    help="CPU self-test of the launcher and routing: a stand-in engine that computes nothing")
    ap.add_argument("--stand-in-step-ms", type=float, default=0.0, help="--stand-in-engine: time per step")
    ap.add_argument("--no-redirect", action="store_true",
                    help="multi-process server: no overflow redirect to the least-loaded worker (LoadBoard)")
    args = ap.parse_args(argv)
    import sys

    if (args.gpus > 1 or args.torchrun) and "WORLD_SIZE" not in os.environ:
        import socket
        import subprocess

        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            mport = so.getsockname()[1]
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", f"--master-port={mport}", "-m", "pocket_tts_amd.serve",
               *(argv if argv is not None else sys.argv[1:])]
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0",
                   PYTHONPATH=os.pathsep.join([os.path.dirname(os.path.dirname(__file__)),
                                               os.environ.get("PYTHONPATH", "")]))
        sys.exit(subprocess.run(cmd, env=env).returncode)
    # the scheduler thread drops the GIL in every engine call; with the default 5 ms switch
    # interval it can wait that long to get it back from the HTTP threads (one engine step is
    # < 1 ms), so hand the GIL over sooner
    sys.setswitchinterval(2e-4)
    if args.stand_in_engine:
        Engine = StandInEngine
    else:
        from .engine import Engine
    engine, rank, world, checksum = _worker_engine(args, Engine)
    voices: dict[str, Voice] = {}
    for spec in args.voice or []:
        name, path = spec.split("=", 1)
        if path.endswith(".npy"):
            voices[name] = engine.voice_from_prompt(np.load(path, allow_pickle=False).astype(np.float32))
        else:  # a WAV voice prompt: resampled to 24 kHz on the GPU, Mimi-encoded (tts_model.rs:446-463)
            from .audio import read_wav

            audio, sr = read_wav(path)
            if audio.shape[0] != 1:
                raise SystemExit(f"voice prompt {path} must be mono")
            voices[name] = engine.voice_from_audio(audio[0], sr)
    if not voices:
        raise SystemExit("at least one --voice NAME=path is required")
    scheduler = BatchScheduler(engine, preview_rows=args.preview_rows)
    service = TTSService(scheduler, voices, default_voice=next(iter(voices)),
                         tokenizer=load_tokenizer(args.tokenizer) if args.tokenizer else None)
    service.worker = {"rank": rank, "world": world, "pid": os.getpid(), "weights_checksum": checksum}
    socks = [_listen_socket(args.host, args.port)]
    board = None
    if world > 1 and not args.no_redirect:  # least-loaded dispatch across the workers (LoadBoard)
        board = LoadBoard(args.port, world, rank, scheduler.max_rows)
        board.publish(0)
        priv = _listen_socket(args.host, 0, reuse_port=False)
        board.set_private_port(priv.getsockname()[1])
        socks.append(priv)
        scheduler.on_load = board.publish
        service.board, service.shared_port = board, args.port
    import uvicorn

    app = create_app(service)
    try:
        uvicorn.Server(uvicorn.Config(app, log_level="warning")).run(sockets=socks)
    finally:
        if board is not None:
            board.close(unlink=rank == 0)


if __name__ == "__main__":
    main()
