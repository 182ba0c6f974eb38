"""The server's reader-thread submit path (serve/server.py VisionAnalysisService._analyze_pipelined with
EngineSession.submit_encoded_handle / collect_handle) on the CPU, through a fake engine: responses in
request order for streaming and lock-step clients, declined and failing frames answered in place, at most
``depth`` frames between the reader and the handler, and every pipeline back in its pool however the stream
ends. The GPU path is tests/test_serve_gpu.py::test_encoded_fast_path_matches_decode_path.
Reference per-frame loop: /root/reference/services/vision_analysis/server.py:113-158."""
import queue
import threading
import time

import pytest

from robotic_discovery_platform_amd.proto import vision as pb
from robotic_discovery_platform_amd.serve.engine import WireResult
from robotic_discovery_platform_amd.serve.server import VisionAnalysisService


class FakePipe:
    """A pipeline whose 'frame' is the colour payload, answered as the response's status."""

    def __init__(self, log):
        self.payload, self.log = None, log

    def collect_encoded(self):
        time.sleep(0.002)  # the GPU
        p = self.payload
        if p.startswith(b"boom"):
            raise RuntimeError("device failure")
        msg = pb.AnalysisResponse(status=p.decode(), mask_coverage=1.0).SerializeToString()
        return WireResult(msg, 0.1, 0.2, 1.0, 0.5)


class FakeSession:
    depth = 2

    def __init__(self, pool_q, log):
        self.q, self.log, self.closed = pool_q, log, False
        self.outstanding = 0
        self.max_outstanding = 0
        self.lock = threading.Lock()

    def submit_encoded_handle(self, color, depth, stop=None):
        if color.startswith(b"declined"):
            return ("d", 1)
        p = self.q.get(timeout=5)
        p.payload = color
        with self.lock:
            self.outstanding += 1
            self.max_outstanding = max(self.max_outstanding, self.outstanding)
        self.log.append(("submit", color))
        return ("t", (p, self.q))

    def submit(self, c, d, tag=None, rgb=False):
        return []

    def drain(self):
        return [(None, ValueError("array path failed"))]

    def close(self):
        self.closed = True


class FakeEngine:
    jpeg, gpu, home_size = True, True, (480, 640)

    def __init__(self, n=4):
        self.q = queue.Queue()
        self.log = []
        for _ in range(n):
            self.q.put(FakePipe(self.log))
        self.sessions = []

    def session(self):
        s = FakeSession(self.q, self.log)
        self.sessions.append(s)
        return s


class Ctx:
    def set_code(self, c):
        self.code = c

    def set_details(self, d):
        self.details = d


@pytest.fixture
def svc(monkeypatch):
    monkeypatch.setenv("RDP_SERVE_READER_SUBMIT", "1")
    eng = FakeEngine()
    s = VisionAnalysisService(eng, None)
    s._decode_color = lambda b: b  # declined frames: "decoded" here, then the (failing) array path
    s._decode_depth = lambda b: b
    assert s._encoded and s.reader_submit
    orig = type(s)._analyze_pipelined
    s.pipelined_calls = 0

    def wrapped(self, it, ctx):
        self.pipelined_calls += 1
        yield from orig(self, it, ctx)
    monkeypatch.setattr(type(s), "_analyze_pipelined", wrapped)
    yield s, eng
    s.close()


def _track_outstanding(eng):
    """Collected frames decrement the session's outstanding count (the pipe goes back to the pool)."""
    orig = FakePipe.collect_encoded

    def collect(self):
        try:
            return orig(self)
        finally:
            for s in eng.sessions:
                with s.lock:
                    s.outstanding -= 1
    return collect


def _req(tag):
    return pb.AnalysisRequest(color_image=pb.Image(data=tag), depth_image=pb.Image(data=b"d"))


def test_streaming_in_order_with_declined_and_failing_frames(svc, monkeypatch):
    s, eng = svc
    monkeypatch.setattr(FakePipe, "collect_encoded", _track_outstanding(eng))
    tags = [b"f0", b"f1", b"declined2", b"f3", b"boom4", b"f5", b"f6"]
    out = [pb.AnalysisResponse.FromString(r if isinstance(r, bytes) else r.SerializeToString())
           for r in s.AnalyzeActuatorPerformance(iter([_req(t) for t in tags]), Ctx())]
    assert s.pipelined_calls == 1
    st = [r.status for r in out]
    assert st[:2] == ["f0", "f1"] and st[3] == "f3" and st[5:] == ["f5", "f6"]
    assert st[2].startswith("error: ValueError") and st[4].startswith("error: RuntimeError")
    assert eng.q.qsize() == 4  # every pipeline back in the pool
    assert eng.sessions[0].max_outstanding <= 2 and eng.sessions[0].closed
    assert s.frame_failures == 2


def test_lockstep_client_does_not_deadlock(svc, monkeypatch):
    s, eng = svc
    got = queue.Queue()

    def lockstep():  # sends frame i + 1 only after response i arrived
        for i in range(6):
            yield _req(b"f%d" % i)
            got.get(timeout=10)

    out = []
    for r in s.AnalyzeActuatorPerformance(lockstep(), Ctx()):
        out.append(pb.AnalysisResponse.FromString(r if isinstance(r, bytes) else r.SerializeToString()).status)
        got.put(1)
    assert out == ["f%d" % i for i in range(6)]
    assert eng.q.qsize() == 4


def test_stream_ending_early_returns_every_pipeline(svc):
    s, eng = svc
    gen = s.AnalyzeActuatorPerformance(iter([_req(b"f%d" % i) for i in range(50)]), Ctx())
    first = [next(gen) for _ in range(3)]
    assert len(first) == 3
    gen.close()  # the client went away: GeneratorExit at the yield
    deadline = time.time() + 5
    while eng.q.qsize() < 4 and time.time() < deadline:  # the reader frees a frame it still held
        time.sleep(0.01)
    assert eng.q.qsize() == 4
    assert eng.sessions[0].closed
