"""BatchEngine's batching state machine on the CPU (serve/engine.py: positions, launcher thread, tickets,
generations, frame rotation), driven through a fake native runner: no GPU, no graphs. The device program
itself is covered by tests/test_serve_batch_gpu.py.

What is pinned here:
* a batch launches once, with every staged position, and its frame rotates back only after every ticket
  is collected;
* the launch policy waits for the active stream count (``target``) and sends a partial batch after
  ``max_wait``;
* a batch whose positions all failed staging is never launched, and its frame is reused at once (a new
  generation: a ticket never reads a stale launch);
* a launch that raises fails every waiting collector and later acquires, instead of hanging them;
* ``hold`` takes every frame and ``unhold`` gives them back.
Reference per-frame body: /root/reference/services/vision_analysis/server.py:116-152."""
import collections
import contextlib
import threading
import time

import pytest
import torch

from robotic_discovery_platform_amd.serve import engine as E


class FakeEvent:
    busy = False  # True: every launched batch still "on the GPU"

    def record(self, stream=None):
        pass

    def query(self):
        return not FakeEvent.busy


class FakeRunner:
    """decode: code per colour payload (b"ok" -> 0, else 3); launch: records (k, n, staged payloads)."""

    def __init__(self, fail_launch=False):
        self.payload = {}
        self.launches = []
        self.fail_launch = fail_launch
        self.lock = threading.Lock()

    def decode(self, k, j, color, depth):
        with self.lock:
            self.payload[(k, j)] = color
        return 0 if color.startswith(b"ok") else 3

    def launch(self, k, n):
        if self.fail_launch:
            raise RuntimeError("injected launch failure")
        with self.lock:
            self.launches.append((k, n, [self.payload[(k, j)] for j in range(n)]))

    def collect_encoded(self, k, j, level, bands):
        with self.lock:
            return self.payload[(k, j)], 1.0, 2.0, 3.0, 0, 0.1

    def drain(self):
        pass


@pytest.fixture(autouse=True)
def no_gpu(monkeypatch):
    monkeypatch.setattr(torch.cuda, "device", lambda *a, **k: contextlib.nullcontext())
    monkeypatch.setattr(torch.cuda, "Event", FakeEvent)


def make(runner, frames=2, positions=4, window_us=200000.0, max_wait_us=5e6, target=None):
    """A BatchEngine with only its batching state (the device program is not built)."""
    be = E.BatchEngine.__new__(E.BatchEngine)
    be.runner, be.nf, be.P, be.lanes = runner, frames, positions, 1
    be.window, be.max_wait = window_us * 1e-6, max_wait_us * 1e-6
    be.lane_stream = [None]
    be.dev = None
    be.target = target
    be._init_batching()  # batching state + the launcher thread
    return be


def submit_n(be, payloads):
    pos = [be._acquire() for _ in payloads]
    return [be.submit_encoded(p, b"d", pos=q) for p, q in zip(payloads, pos)]


def test_one_launch_per_batch_and_rotation_after_collect():
    r = FakeRunner()
    be = make(r, frames=2)
    try:
        tick = submit_n(be, [b"ok0", b"ok1", b"ok2"])
        got = [be.collect_encoded(t).payload for _, t in tick]
        assert got == [b"ok0", b"ok1", b"ok2"]
        assert r.launches == [(tick[0][1][0], 3, [b"ok0", b"ok1", b"ok2"])]
        assert dict(be.batch_sizes) == {3: 1}
        with be._cv:
            assert sorted(be._free) == [0, 1] and be._refs == [0, 0]
    finally:
        be.close()


def test_target_waits_for_every_active_stream_then_max_wait():
    r = FakeRunner()
    be = make(r, frames=2, window_us=300000.0, max_wait_us=800000.0, target=lambda: 3)
    try:
        pair = submit_n(be, [b"ok0", b"ok1"])
        time.sleep(0.05)  # a target of 3 streams: the pair waits for the third frame ...
        assert r.launches == []
        t0 = time.perf_counter()
        t3 = be.submit_encoded(b"ok2", b"d")[1]  # ... which launches the batch at once
        assert be.collect_encoded(t3).payload == b"ok2"
        assert time.perf_counter() - t0 < 0.25
        assert [n for _, n, _ in r.launches] == [3]
        assert [be.collect_encoded(t).payload for _, t in pair] == [b"ok0", b"ok1"]
        # a lone frame while a batch is still on the GPU: past its window it keeps waiting for more
        # frames, and goes after max_wait
        FakeEvent.busy = True
        t0 = time.perf_counter()
        t = be.submit_encoded(b"ok3", b"d")[1]
        assert be.collect_encoded(t).payload == b"ok3"
        assert time.perf_counter() - t0 >= 0.7
        assert [n for _, n, _ in r.launches] == [3, 1]
    finally:
        FakeEvent.busy = False
        be.close()


def test_all_void_batch_is_not_launched_and_frame_reused():
    r = FakeRunner()
    be = make(r, frames=1)
    try:
        first = submit_n(be, [b"ok-a", b"ok-b"])
        assert [be.collect_encoded(t).payload for _, t in first] == [b"ok-a", b"ok-b"]
        void = submit_n(be, [b"bad"] * 4)  # a full frame: the next acquire waits for it to close
        assert all(code == 3 for code, _ in void)
        second = submit_n(be, [b"ok-c", b"ok-d"])
        assert second[0][1][2] == first[0][1][2] + 2  # same frame, a later generation
        assert [be.collect_encoded(t).payload for _, t in second] == [b"ok-c", b"ok-d"]
        assert [n for _, n, _ in r.launches] == [2, 2]  # the void batch never ran
    finally:
        be.close()


def test_launch_failure_fails_collectors_and_acquires():
    r = FakeRunner(fail_launch=True)
    be = make(r, frames=2)
    try:
        (code, t), = submit_n(be, [b"ok0"])
        assert code == 0
        with pytest.raises(RuntimeError, match="injected launch failure"):
            be.collect_encoded(t)
        with pytest.raises(RuntimeError, match="launch failed"):
            be._acquire()
    finally:
        be.close()


def test_hold_takes_every_frame_until_unhold():
    r = FakeRunner()
    be = make(r, frames=2)
    try:
        tick = submit_n(be, [b"ok0"])
        held = threading.Event()

        def holder():
            be.hold()
            held.set()

        th = threading.Thread(target=holder, daemon=True)
        th.start()
        time.sleep(0.05)
        assert not held.is_set()  # frame 0's result is not collected yet
        be.collect_encoded(tick[0][1])
        assert held.wait(5.0)
        assert be._acquire(block=False) is None
        be.unhold()
        assert be._acquire(block=False) is not None
    finally:
        be.close()
