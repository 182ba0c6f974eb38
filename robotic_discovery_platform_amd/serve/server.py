"""VisionAnalysisService gRPC server (``evofab.vision``, stream -> stream).

Behaviour of ``/root/reference/services/vision_analysis/server.py:22-183``:
  * resources: model from the registry URI (default ``models:/Actuator-Segmenter/latest``,
    ``@alias`` also accepted), intrinsics ``mtx`` + optional ``depth_scale`` (default 0.001) from
    ``ml/configs/calibration_data.npz``; startup aborts if any is missing          (:74-99,166-170)
  * per request: decode JPEG colour + 16-bit PNG depth, mask/curvature, response with mean/max
    curvature, 100 spline points and the PNG mask (u8 {0,255}) at frame size       (:116-152)
  * per-frame CSV ``timestamp,mean_curvature,max_curvature,mask_coverage_percent`` (:68-72,146-150)
  * any exception: ``StatusCode.INTERNAL`` + details + one empty response         (:154-158)
  * ``ThreadPoolExecutor(max_workers=10)`` on ``[::]:50051``                       (:172-179)

Differences: ``status``, ``mask_coverage`` and ``proc_time_ms`` are populated (a
wire-compatible superset); the CSV writer is locked and keeps its handle open (the reference appends
from 10 threads without a lock); colour and depth are decoded concurrently on a codec thread pool,
up to ``prefetch`` frames ahead, so host codecs overlap the device program; the model can hot-reload
when a registry alias moves.
"""
from __future__ import annotations

import collections
import logging
import os
import queue
import threading
import time
from concurrent import futures
from typing import Optional

import numpy as np
import torch

from ..config import ServeConfig
from ..data.image_io import decode_image, encode_png
from ..data.jpeg import decode_coefs
from ..proto import vision as pb
from ..utils import trace
from .engine import RESP_PNG_BANDS, RESP_PNG_LEVEL, EnginePool, EngineSession, WireResult, _is_native

log = logging.getLogger(__name__)

CSV_HEADER = "timestamp,mean_curvature,max_curvature,mask_coverage_percent\n"


class MetricsLog:
    """Thread-safe per-frame metrics CSV (same header/row format as the reference)."""

    def __init__(self, path: str):
        self.path = path
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        try:  # exactly one writer creates the file and its header (server worker processes race here)
            fd = os.open(path, os.O_WRONLY | os.O_APPEND | os.O_CREAT | os.O_EXCL, 0o644)
        except FileExistsError:
            pass
        else:
            with os.fdopen(fd, "w") as f:
                f.write(CSV_HEADER)
        self._f = open(path, "a", buffering=1)
        self._lock = threading.Lock()

    def write(self, mean_k: float, max_k: float, coverage: float, ts: Optional[float] = None) -> None:
        line = f"{time.time() if ts is None else ts},{mean_k},{max_k},{coverage}\n"
        with self._lock:
            self._f.write(line)

    def close(self) -> None:
        with self._lock:
            self._f.close()


def load_resources(cfg: ServeConfig, device: Optional[torch.device] = None):
    """(model, intrinsics, depth_scale, version) or Nones, logging the reason like the reference."""
    from ..camera import load_calibration
    from ..mlstore import pytorch as mlpt
    from ..mlstore.store import FileStore
    model = K = ds = version = None
    try:
        model = mlpt.load_model(cfg.model_uri, map_location=device, backend=cfg.backend,
                                tracking_uri=cfg.mlruns_dir)
        version = registry_version(FileStore(cfg.mlruns_dir), cfg.model_uri)
        log.info("segmentation model '%s' loaded (version %s)", cfg.model_uri, version)
    except Exception as e:
        log.error("FATAL: failed to load model %s: %s", cfg.model_uri, e)
        return None, None, None, None
    if not os.path.exists(cfg.calib_file):
        log.error("FATAL: calibration data not found at '%s'", cfg.calib_file)
        return model, None, None, version
    try:
        K, _, ds = load_calibration(cfg.calib_file, cfg.default_depth_scale)
    except Exception as e:
        log.error("FATAL: failed to load intrinsics: %s", e)
        return model, None, None, version
    return model, K, ds, version


def registry_version(store, uri: str) -> Optional[str]:
    """The concrete version a ``models:/`` URI currently points at (None for run URIs)."""
    if not uri.startswith("models:/"):
        return None
    name, _, ref = uri[len("models:/"):].partition("/")
    if "@" in name:
        name, alias = name.split("@", 1)
        return str(store.get_model_version_by_alias(name, alias).version)
    if ref in ("", "latest"):
        vs = store.search_model_versions(name)
        return str(max(int(v.version) for v in vs)) if vs else None
    if ref.isdigit():
        return ref
    vs = store.get_latest_versions(name, stages=[ref])
    return str(vs[0].version) if vs else None


class VisionAnalysisService(pb.VisionAnalysisServiceServicer):
    """Per-stream pipeline: decode (codec pool, runs ahead) -> engine session (double-buffered on one
    GPU replica) -> response encode (codec pool), responses in request order.

    Failure semantics: the reference ends the stream with ``StatusCode.INTERNAL`` + one empty
    response on any exception (server.py:154-158); that stays the behaviour for transport errors and
    with ``frame_errors="abort"``. With the default ``frame_errors="degrade"`` a frame that cannot be
    decoded or analysed (truncated PNG, corrupt JPEG, size mismatch, ...) gets a response with
    ``status="error: ..."`` and zero curvature, and the stream goes on. ``faults`` is an optional
    ``FaultInjector`` (tests / chaos runs) that corrupts requests before decoding.
    """

    def __init__(self, engine: EnginePool, metrics: Optional[MetricsLog] = None, prefetch: int = 4,
                 decode_workers: int = 8, frame_errors: str = "degrade", faults=None):
        self.engine = engine
        self.metrics = metrics
        self.prefetch = prefetch
        self.frame_errors = frame_errors
        self.faults = faults
        self.frames = 0
        self.frame_failures = 0
        self._stats_lock = threading.Lock()
        self.queue_ms: "collections.deque" = collections.deque(maxlen=4096)  # request read -> processing start
        self.proc_ms: "collections.deque" = collections.deque(maxlen=4096)  # processing start -> response ready
        # per-stage times of every frame (ms; latency_stats() reports p50 / p99): decode_color /
        # decode_depth (codec pool), submit (engine staging + graph launch, handler thread), gpu (the
        # frame's device time), respond (mask PNG + response message, codec pool), hold (response
        # ready -> handed to gRPC)
        self.stage_ms = {k: collections.deque(maxlen=4096)
                         for k in ("decode_color", "decode_depth", "submit", "gpu", "respond", "hold")}
        # shared host-codec pool: JPEG / 16-bit PNG decodes release the GIL, so colour and depth of a
        # frame, and up to `prefetch` frames of a stream, decode concurrently
        self._pool = futures.ThreadPoolExecutor(max_workers=decode_workers, thread_name_prefix="rdp-decode")
        # colour frames of a GPU engine built for it: JPEG entropy decode only (pinned coefficients),
        # the pixel stage runs in the frame graph (data/jpeg.py)
        self._gpu_jpeg = bool(getattr(engine, "jpeg", False))
        self._pin = bool(getattr(engine, "gpu", False))  # pinned coefficient buffers: GPU engines only
        # whole frames natively (EngineSession.submit_encoded): the request bytes go to a pipeline that
        # decodes, launches, waits and encodes the response without the interpreter lock; this thread
        # only moves bytes. Frames that path declines take the decode path below.
        self._encoded = self._gpu_jpeg and self._pin and hasattr(engine, "home_size")
        # RDP_SERVE_RAW=1: requests arrive as their serialized bytes (proto/vision.py registers the handler
        # without a deserializer) and the native path reads the two image payloads in place. Measured slower
        # than gRPC's own parse (e2e 1 stream 1,932 / 2,034 vs 2,193 / 2,230 FPS, 4 streams 3,645 / 3,333 vs
        # 3,729 / 3,566; profiles/serve_e2e.md round 6), so off by default (fault injection needs the fields)
        self.raw_requests = self._encoded and faults is None and os.environ.get("RDP_SERVE_RAW", "0") == "1"
        # encoded frames submitted by the stream's reader thread while the client streams (decode + launch of
        # frame i + 1 overlaps the collection of frame i: _analyze_pipelined); RDP_SERVE_READER_SUBMIT=0: the
        # handler submits -- the default of multi-process servers (_serve_workers)
        self.reader_submit = os.environ.get("RDP_SERVE_READER_SUBMIT", "1") != "0"
        try:
            from ..ops import native
            self._encode = getattr(native(build_if_missing=False), "encode_response", None)
        except Exception:  # pragma: no cover - no extension: message path
            self._encode = None

    def _decode_color(self, data: bytes):
        t = time.perf_counter()
        out = None
        if self._gpu_jpeg and data[:2] == b"\xff\xd8":
            out = decode_coefs(data, parallel=True, pin=self._pin)
        if out is None:
            out = decode_image(data, True, "RGB")  # no BGR flip: the engine takes RGB
        self.stage_ms["decode_color"].append((time.perf_counter() - t) * 1e3)
        return out

    def _decode_depth(self, data: bytes):
        t = time.perf_counter()
        out = self._as_u16(decode_image(data, False))
        self.stage_ms["decode_depth"].append((time.perf_counter() - t) * 1e3)
        return out

    def _decoded(self, request_iterator):
        """Yield (t_read, colour, depth future, error, more) in request order; decoding runs ahead on
        the codec pool. ``error`` is the colour decode exception of a bad frame (colour None then; a
        depth decode error surfaces as that frame's result); ``more()`` tells whether the client has
        already sent the next frame."""
        q: "queue.Queue" = queue.Queue(maxsize=self.prefetch)
        END = object()
        stop = threading.Event()  # the handler is gone (stream ended early): the reader must not block

        def put(item) -> bool:
            while not stop.is_set():
                try:
                    q.put(item, timeout=0.1)
                    return True
                except queue.Full:
                    continue
            return False

        def reader():
            try:
                for i, req in enumerate(request_iterator):
                    t = time.perf_counter()
                    if isinstance(req, (bytes, bytearray)):  # raw_requests: the serialized message
                        if not put((t, _Raw(req), None, None)):
                            return
                        continue
                    cb, db = req.color_image.data, req.depth_image.data
                    if self.faults is not None:
                        cb, db = self.faults.corrupt_request(i, cb, db)
                    if self._encoded:  # decoded natively by the pipeline (or on demand, see the handler)
                        if not put((t, cb, db, None)):
                            return
                        continue
                    fc = self._pool.submit(self._decode_color, cb)
                    fd = self._pool.submit(self._decode_depth, db)
                    if not put((t, fc, fd, None)):
                        return
            except Exception as e:  # surface transport errors in the handler thread
                put((None, None, None, e))
            put(END)

        th = threading.Thread(target=reader, daemon=True)
        th.start()
        try:
            while True:
                item = q.get()
                if item is END:
                    return
                if item[3] is not None:
                    raise item[3]
                t, fc, fd, _ = item
                if isinstance(fc, (bytes, _Raw)):  # encoded frame: (colour bytes, depth bytes) / raw request
                    yield t, fc, fd, None, lambda: q.qsize() > 0
                    continue
                try:
                    color, err = fc.result(), None
                except Exception as e:
                    color, err = None, e
                yield t, color, fd, err, lambda: q.qsize() > 0
        finally:
            stop.set()

    def close(self) -> None:
        """Stop the codec pool (its threads must not outlive the gRPC server at interpreter exit)."""
        self._pool.shutdown(wait=True)

    def analyze_frame(self, color: np.ndarray, depth: np.ndarray, t0: Optional[float] = None):
        t0 = time.perf_counter() if t0 is None else t0
        resp, r = self._respond(self._process(color, depth), (t0, t0))
        self._log(r)
        return resp

    @staticmethod
    def _as_u16(depth: np.ndarray) -> np.ndarray:
        return depth if depth.dtype == np.uint16 else depth.astype(np.uint16)

    def _process(self, color: np.ndarray, depth: np.ndarray):
        return self.engine.process(color, self._as_u16(depth))

    def _log(self, r):
        if self.metrics is not None and r is not None:
            if isinstance(r, WireResult):
                self.metrics.write(r.mean_curvature, r.max_curvature, r.coverage)
            else:
                c = r.curvature
                self.metrics.write(c.mean_curvature, c.max_curvature, r.coverage)
        self.frames += 1

    def _wire_ready(self, r: "WireResult", t):
        """A natively served frame: the response bytes exist already; bookkeeping only."""
        t_read, t_start = t
        now = time.perf_counter()
        with self._stats_lock:
            self.queue_ms.append((t_start - t_read) * 1e3)
            self.proc_ms.append((now - t_start) * 1e3)
        self.stage_ms["gpu"].append(r.gpu_ms)
        return r.payload, r, now

    def _respond_timed(self, r, t):
        t0 = time.perf_counter()
        resp, r = self._respond_wire(r, t)
        t1 = time.perf_counter()
        self.stage_ms["respond"].append((t1 - t0) * 1e3)
        if r is not None and "gpu_ms" in r.timings:
            self.stage_ms["gpu"].append(r.timings["gpu_ms"])
        return resp, r, t1

    def _respond_wire(self, r, t):
        """Streaming form of ``_respond``: the AnalysisResponse as wire bytes, mask PNG and message
        encoded natively without the GIL (csrc/serve_runtime.cpp encode_response; byte-identical to the
        message path, tests/test_serve_cpu.py). Error frames, and builds without the extension, take the
        message path."""
        if isinstance(r, Exception) or self._encode is None:
            return self._respond(r, t)
        c = r.curvature
        pts = r.points
        if pts is None and c.spline_points:
            pts = np.array([(p.x, p.y, p.z) for p in c.spline_points], np.float64)
        t_read, t_start = t
        now = time.perf_counter()
        payload = self._encode(c.mean_curvature, c.max_curvature, pts, c.status, r.mask, r.coverage,
                               (now - t_start) * 1e3, RESP_PNG_LEVEL, RESP_PNG_BANDS)
        with self._stats_lock:
            self.queue_ms.append((t_start - t_read) * 1e3)
            self.proc_ms.append((now - t_start) * 1e3)
        return payload, r

    def _respond(self, r, t):
        """FrameResult (or the frame's exception) -> AnalysisResponse; runs on the codec pool when
        streaming. ``t`` = (request read, processing start): proc_time_ms is the server's processing
        time of this frame (decode wait excluded), the queueing before it is kept separately."""
        t_read, t_start = t
        if isinstance(r, Exception):
            resp = pb.AnalysisResponse(status=f"error: {type(r).__name__}: {r}"[:200])
            r = None
        else:
            c = r.curvature
            resp = pb.AnalysisResponse(mean_curvature=c.mean_curvature, max_curvature=c.max_curvature,
                                       status=c.status, mask_coverage=r.coverage)
            if c.spline_points:
                resp.spline_points.extend([pb.Point3D(x=p.x, y=p.y, z=p.z) for p in c.spline_points])
            resp.mask = encode_png(r.mask * np.uint8(255), compress_level=RESP_PNG_LEVEL, bands=RESP_PNG_BANDS)
        now = time.perf_counter()
        resp.proc_time_ms = (now - t_start) * 1e3
        with self._stats_lock:
            self.queue_ms.append((t_start - t_read) * 1e3)
            self.proc_ms.append((now - t_start) * 1e3)
        return resp, r

    def latency_stats(self) -> dict:
        with self._stats_lock:
            q, p = list(self.queue_ms), list(self.proc_ms)
            st = {k: list(v) for k, v in self.stage_ms.items()}
        pct = (lambda v, k: float(np.percentile(v, k)) if v else float("nan"))
        out = {"queue_p50_ms": pct(q, 50), "proc_p50_ms": pct(p, 50), "proc_p99_ms": pct(p, 99),
               "frames": self.frames, "frame_failures": self.frame_failures}
        for k, v in st.items():
            out[f"{k}_p50_ms"] = pct(v, 50)
            out[f"{k}_p99_ms"] = pct(v, 99)
        return out

    def AnalyzeActuatorPerformance(self, request_iterator, context):
        """Responses leave in request order; one that is ready -- or any, when the client has not
        sent the next frame yet (lock-step clients) -- is never held back."""
        import grpc
        if self._encoded and self.reader_submit and self.faults is None and not self.raw_requests:
            yield from self._analyze_pipelined(request_iterator, context)
            return
        log.info("new analysis stream")
        inflight: "collections.deque" = collections.deque()  # encode futures, request order
        sess = self.engine.session()
        times = {}

        def encode(results):
            for tag, r in results:
                if isinstance(r, Exception):
                    if self.frame_errors == "abort":
                        raise r
                    self.frame_failures += 1
                    log.warning("frame failed (%s: %s): degraded response", type(r).__name__, r)
                if isinstance(r, WireResult):
                    inflight.append(_Ready(self._wire_ready(r, times.pop(tag))))
                else:
                    inflight.append(self._pool.submit(self._respond_timed, r, times.pop(tag)))

        def ready(force: bool):
            while inflight and (force or inflight[0].done() or len(inflight) > self.prefetch):
                resp, r, t_ready = inflight.popleft().result()
                self._log(r)
                self.stage_ms["hold"].append((time.perf_counter() - t_ready) * 1e3)
                yield resp

        frames = self._decoded(request_iterator)
        try:
            for i, (t_read, color, depth, err, more) in enumerate(frames):
                t_start = time.perf_counter()
                times[i] = (t_read, t_start)
                if isinstance(color, (bytes, _Raw)):  # encoded frame: natively decoded + launched by a pipeline
                    with trace.range("serve.rpc.frame"):
                        if isinstance(color, _Raw):
                            done, code = sess.submit_request(color.raw, tag=i)
                            if code != 0:  # not taken natively: the message's fields for the paths below
                                req = pb.AnalysisRequest.FromString(color.raw)
                                color, depth = req.color_image.data, req.depth_image.data
                        else:
                            done, code = sess.submit_encoded(color, depth, tag=i)
                        encode(done)
                        if code != 0:  # a frame that path declines: decode here, then the array path
                            try:
                                c, d = self._decode_color(color), self._decode_depth(depth)
                            except Exception as e:
                                encode(sess.drain())
                                encode([(i, e)])
                            else:
                                encode(sess.submit(c, d, tag=i, rgb=True))
                        self.stage_ms["submit"].append((time.perf_counter() - t_start) * 1e3)
                    if not more():
                        encode(sess.drain())
                elif err is not None:
                    encode(sess.drain())  # keep request order: older frames first
                    encode([(i, err)])
                else:
                    with trace.range("serve.rpc.frame"):
                        # colour half enqueued now, depth half when its PNG is inflated
                        done = sess.submit(color, depth, tag=i, rgb=True)
                        self.stage_ms["submit"].append((time.perf_counter() - t_start) * 1e3)
                        encode(done)
                    if not more():  # lock-step client: finish this frame now
                        encode(sess.drain())
                yield from ready(force=not more())
            encode(sess.drain())
            yield from ready(force=True)
        except Exception as e:
            log.error("unhandled exception during analysis: %s", e)
            context.set_code(grpc.StatusCode.INTERNAL)
            context.set_details(f"Internal error during analysis: {e}")
            yield pb.AnalysisResponse()
        finally:
            # however the stream ends (normal end, client cancel -> GeneratorExit at a yield, transport
            # error, abort), the session's in-flight pipelines go back to the pool and the reader stops
            sess.close()
            frames.close()


    def _analyze_pipelined(self, request_iterator, context):
        """The native whole-frame path with the submit on the stream's reader thread
        (``EngineSession.submit_encoded_handle``) while the client streams: a frame that arrives while
        earlier frames of the stream are still unanswered is decoded and launched by the reader, so frame
        i + 1 decodes while this thread collects frame i (at most ``depth`` frames between the two). A frame
        that arrives when every earlier one is answered (lock-step clients) is submitted by this thread, as
        in the handler path. Frames the native path declines are decoded here and served through the array
        path, in order. Each response leaves as soon as its frame is collected, in request order."""
        import grpc
        log.info("new analysis stream")
        sess = self.engine.session()
        items: "queue.Queue" = queue.Queue()
        END = object()
        lk = threading.Lock()
        state = {"stopped": False, "pending": 0}  # pending: frames handed over, not yet answered
        stop = threading.Event()
        slots = threading.Semaphore(max(1, sess.depth))

        def hand_over(item) -> bool:  # False once the handler is gone (the caller then frees the frame)
            with lk:
                if not state["stopped"]:
                    items.put(item)
                    state["pending"] += 1
                    return True
            return False

        def submit(cb, db, t_start):
            try:
                kv = sess.submit_encoded_handle(cb, db, stop)
            except Exception as e:
                kv = ("e", e)
            self.stage_ms["submit"].append((time.perf_counter() - t_start) * 1e3)
            return kv

        def reader():
            try:
                for i, req in enumerate(request_iterator):
                    t_read = time.perf_counter()
                    while not slots.acquire(timeout=0.05):
                        if stop.is_set():
                            return
                    cb, db = req.color_image.data, req.depth_image.data
                    t_start = time.perf_counter()
                    with lk:
                        streaming = state["pending"] > 0
                    if streaming:
                        kind, val = submit(cb, db, t_start)
                    else:
                        kind, val = "r", None  # the handler submits it (no extra hop on a lock-step frame)
                    if not hand_over((i, t_read, t_start, kind, val, cb, db)):
                        if kind == "t":
                            EngineSession.collect_handle(val)
                        return
            except Exception as e:  # transport errors surface in the handler thread
                hand_over((None, None, None, "x", e, None, None))
            hand_over(END)

        threading.Thread(target=reader, daemon=True, name="rdp-stream-reader").start()
        try:
            while True:
                it = items.get()
                if it is END:
                    break
                i, t_read, t_start, kind, val, cb, db = it
                if kind == "x":
                    raise val
                if kind == "r":
                    kind, val = submit(cb, db, t_start)
                try:
                    if kind == "t":
                        results = [(i, EngineSession.collect_handle(val))]
                    elif kind == "e":
                        results = [(i, val)]
                    else:  # declined by the native path: decoded here, the array path
                        try:
                            c, d = self._decode_color(cb), self._decode_depth(db)
                        except Exception as e:
                            results = [(i, e)]
                        else:
                            results = sess.submit(c, d, tag=i, rgb=True) + sess.drain()
                finally:
                    slots.release()
                for _, r in results:
                    yield self._respond_one(r, (t_read, t_start))
                with lk:  # answered (gRPC asks for the next response once this one is sent)
                    state["pending"] -= 1
        except Exception as e:
            log.error("unhandled exception during analysis: %s", e)
            context.set_code(grpc.StatusCode.INTERNAL)
            context.set_details(f"Internal error during analysis: {e}")
            yield pb.AnalysisResponse()
        finally:
            # however the stream ends: the reader hands nothing over any more, and the frames it already
            # handed over give their pipelines / batch positions back
            stop.set()
            with lk:
                state["stopped"] = True
            while True:
                try:
                    it = items.get_nowait()
                except queue.Empty:
                    break
                if it is not END and it[3] == "t":
                    EngineSession.collect_handle(it[4])
            sess.close()

    def _respond_one(self, r, t):
        """One collected frame (WireResult, FrameResult or its exception) -> the response, logged."""
        if isinstance(r, Exception):
            if self.frame_errors == "abort":
                raise r
            self.frame_failures += 1
            log.warning("frame failed (%s: %s): degraded response", type(r).__name__, r)
        if isinstance(r, WireResult):
            resp, r2, t_ready = self._wire_ready(r, t)
        else:
            resp, r2, t_ready = self._respond_timed(r, t)
        self._log(r2)
        self.stage_ms["hold"].append((time.perf_counter() - t_ready) * 1e3)
        return resp


class _Raw:
    """A request still in its serialized form (the native path parses it itself)."""
    __slots__ = ("raw",)

    def __init__(self, raw):
        self.raw = bytes(raw)


class _Ready:
    """A response that needs no more work, in the handler's queue of pending futures."""
    __slots__ = ("_v",)

    def __init__(self, v):
        self._v = v

    def done(self) -> bool:
        return True

    def result(self):
        return self._v


class ModelWatcher(threading.Thread):
    """Hot reload: poll the registry; when the URI resolves to a new version, copy the weights in place."""

    def __init__(self, cfg: ServeConfig, model, engine: EnginePool, version: Optional[str], period_s: float = 5.0):
        super().__init__(daemon=True)
        self.cfg, self.model, self.engine, self.version, self.period = cfg, model, engine, version, period_s
        self.stop_evt = threading.Event()
        self.reloads = 0

    def check_once(self) -> bool:
        from ..mlstore import pytorch as mlpt
        from ..mlstore.store import FileStore
        uri = self.cfg.model_uri
        if self.cfg.hot_reload_alias:
            name = uri[len("models:/"):].split("/")[0].split("@")[0]
            uri = f"models:/{name}@{self.cfg.hot_reload_alias}"
        try:
            v = registry_version(FileStore(self.cfg.mlruns_dir), uri)
        except Exception:
            return False
        if v is None or v == self.version:
            return False
        _, sd = mlpt.load_state(uri, self.cfg.mlruns_dir)
        with self.engine.exclusive() as pipelines:
            self.engine.load_state_dict(sd)  # every per-GPU replica
            self.engine.refresh_weights(pipelines)
            if torch.cuda.is_available():
                torch.cuda.synchronize()
        log.info("hot-reloaded %s: version %s -> %s", uri, self.version, v)
        self.version = v
        self.reloads += 1
        return True

    def run(self):
        while not self.stop_evt.wait(self.period):
            self.check_once()


def serving_devices(spec: str, default: Optional[torch.device] = None):
    """``ServeConfig.devices``: "" -> [default], "all" -> every visible GPU, "0,2" -> those GPUs."""
    spec = (spec or "").strip()
    if not spec:
        return None if default is None else [default]
    if spec == "all":
        return [torch.device("cuda", i) for i in range(torch.cuda.device_count())]
    return [torch.device(d) if not d.strip().isdigit() else torch.device("cuda", int(d)) for d in spec.split(",")]


def build_server(cfg: ServeConfig, device: Optional[torch.device] = None, pool_size: Optional[int] = None,
                 port: Optional[int] = None, faults=None):
    """Create (server, service, watcher, bound_port); None if resources are missing (reference abort)."""
    import grpc
    devices = serving_devices(cfg.devices)
    if devices and device is None:
        device = devices[0]
    model, K, ds, version = load_resources(cfg, device)
    if model is None or K is None or ds is None:
        log.error("FATAL: could not load all required resources")
        return None
    metrics = MetricsLog(cfg.metrics_log)
    engine = EnginePool(model, K, ds, n=pool_size or cfg.replicas_per_device, threshold=cfg.mask_threshold,
                        graph=cfg.graph, size=cfg.model_img_size, devices=devices, rgb=True,
                        jpeg=cfg.gpu_jpeg and _is_native(model))
    service = VisionAnalysisService(engine, metrics, frame_errors=cfg.frame_errors, faults=faults)
    server = grpc.server(futures.ThreadPoolExecutor(max_workers=cfg.max_workers))
    pb.add_VisionAnalysisServiceServicer_to_server(service, server)
    bound = server.add_insecure_port(f"{cfg.host}:{cfg.port if port is None else port}")
    watcher = None
    if cfg.hot_reload_alias:
        watcher = ModelWatcher(cfg, model, engine, version)
    freeze_heap()
    return server, service, watcher, bound


def freeze_heap() -> None:
    """Once the long-lived objects exist (model, engine, graphs, gRPC server): move them out of the
    cyclic collector's generations (``gc.freeze``), so a collection triggered by per-frame allocations
    walks only the young objects instead of the whole torch / gRPC heap -- a full pass over it stalled
    the handler threads for milliseconds, the largest single source of slow frames
    (profiles/serve_tail.md)."""
    import gc
    gc.collect()
    gc.freeze()


def serve(cfg: Optional[ServeConfig] = None, block: bool = True):
    """Run the service. ``cfg.workers`` > 1: that many server processes (spawned before anything
    touches the GPU) bind the same port with SO_REUSEPORT -- the kernel spreads client connections
    over them -- each with its own engine replica and its own interpreter lock; the per-frame Python
    work of one process caps it at ~1,500-1,800 frames/s (profiles/serve_e2e.md). ``block``: wait for
    the workers to exit (else return the worker processes)."""
    cfg = cfg or ServeConfig()
    if cfg.workers > 1:
        return _serve_workers(cfg, block)
    from .faults import from_env
    out = build_server(cfg, faults=from_env())
    if out is None:
        return None
    server, service, watcher, port = out
    server.start()
    if watcher is not None:
        watcher.start()
    log.info("VisionAnalysisService listening on %s:%d", cfg.host, port)
    if block:
        server.wait_for_termination()
    return server, service, watcher, port


def _worker_main(cfg: ServeConfig) -> None:
    import dataclasses
    serve(dataclasses.replace(cfg, workers=1), block=True)


def _serve_workers(cfg: ServeConfig, block: bool = True):
    import multiprocessing as mp
    if cfg.port == 0:
        raise ValueError("workers > 1 need a fixed port (every worker binds it with SO_REUSEPORT)")
    ctx = mp.get_context("spawn")  # fresh interpreters: the parent never initialises the GPU
    MetricsLog(cfg.metrics_log).close()  # the CSV and its header exist before any worker appends
    # several server processes on one host: the handler submit (the reader-thread submit measured 8-22 %
    # slower with 2 processes x 2 streams: more concurrent decodes oversubscribe the host's cores;
    # profiles/serve_e2e.md round 6), unless set explicitly
    os.environ.setdefault("RDP_SERVE_READER_SUBMIT", "0")
    procs = [ctx.Process(target=_worker_main, args=(cfg,), name=f"rdp-serve-{i}", daemon=False)
             for i in range(cfg.workers)]
    for p in procs:
        p.start()
    log.info("VisionAnalysisService: %d worker processes on %s:%d", cfg.workers, cfg.host, cfg.port)
    if not block:
        return procs
    try:
        for p in procs:
            p.join()
    except KeyboardInterrupt:
        for p in procs:
            p.terminate()
        for p in procs:
            p.join()
    return [p.exitcode for p in procs]
