"""Host watchdog over natively issued RCCL collectives (parallel/watchdog.py), failure paths on CPU with
a fake communicator: an asynchronous RCCL error and a step whose collectives never complete must both
abort the communicator and end the process non-zero with a rank-tagged message; healthy steps must not.
Also the DDP emulation spec / stream-mode selection used to choose the world > 1 issue stream."""
import os
import subprocess
import sys
import threading
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _Ev:
    def __init__(self, done=False):
        self.done = done

    def query(self):
        return self.done


class _Comm:
    def __init__(self):
        self.code, self.aborted = 0, 0

    def poll(self):
        return (self.code, "remote process exited" if self.code else "")

    def abort(self):
        self.aborted += 1


def _wd(comm, timeout=5.0, rank=3):
    from robotic_discovery_platform_amd.parallel.watchdog import CommWatchdog
    got = []
    done = threading.Event()

    def fail(msg):
        got.append(msg)
        done.set()
    return CommWatchdog(comm.poll, comm.abort, timeout=timeout, period=0.02, rank=rank, on_fail=fail), got, done


def test_healthy_steps_never_fail():
    comm = _Comm()
    wd, got, done = _wd(comm)
    evs = [_Ev() for _ in range(5)]
    for e in evs:
        wd.arm(e)
    time.sleep(0.1)
    for e in evs:
        e.done = True
    time.sleep(0.1)
    assert wd.pending() == 0 and not got and comm.aborted == 0
    wd.close()


def test_async_error_aborts_rank_tagged():
    comm = _Comm()
    wd, got, done = _wd(comm, rank=5)
    wd.arm(_Ev())
    time.sleep(0.05)
    assert not got
    comm.code = 6  # ncclRemoteError
    assert done.wait(2.0)
    assert got[0].startswith("[rank 5]") and "RCCL error 6" in got[0] and "remote process exited" in got[0]
    assert comm.aborted == 1
    wd.close()


def test_stalled_step_times_out():
    comm = _Comm()
    wd, got, done = _wd(comm, timeout=0.2, rank=1)
    wd.arm(_Ev(done=True))  # a finished step ahead of the stuck one is dropped, not timed
    wd.arm(_Ev(done=False))
    assert done.wait(3.0)
    assert got[0].startswith("[rank 1]") and "still incomplete" in got[0] and comm.aborted == 1
    wd.close()


def test_arm_is_bounded():
    comm = _Comm()
    wd, got, done = _wd(comm)
    first = _Ev()
    wd.arm(first)
    for _ in range(200):
        wd.arm(_Ev())
    assert wd.pending() == wd.max_armed and wd._armed[0][1] is first
    wd.close()


def test_default_failure_exits_process_nonzero():
    code = ("import time, sys; sys.path.insert(0, %r)\n"
            "from robotic_discovery_platform_amd.parallel.watchdog import CommWatchdog\n"
            "class E:\n    def query(self): return False\n"
            "wd = CommWatchdog(lambda: (0, ''), None, timeout=0.2, period=0.02, rank=2)\n"
            "wd.arm(E())\ntime.sleep(10)\nprint('not reached')\n" % ROOT)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    from robotic_discovery_platform_amd.parallel.watchdog import EXIT_CODE
    assert r.returncode == EXIT_CODE, (r.returncode, r.stderr)
    assert "[rank 2] RDP comm watchdog" in r.stderr and "not reached" not in r.stdout


def test_emulate_spec_and_model():
    from robotic_discovery_platform_amd.parallel.ddp import emulate_spec, ring_allreduce_us
    assert emulate_spec("") is None
    assert emulate_spec("8:150") == (8, 150.0, 16, 15.0, 0.0)
    assert emulate_spec("4:300:32:5") == (4, 300.0, 32, 5.0, 0.0)
    assert emulate_spec("8:150:16:15:3") == (8, 150.0, 16, 15.0, 3.0)
    for bad in ("8", "1:100", "8:0", "8:100:0", "8:150:16:15:-1"):
        with pytest.raises(ValueError):
            emulate_spec(bad)
    # 69 MB fp32 gradients over 8 ranks at 150 GB/s: 2 * 7/8 * 69e6 / 150e9 s = 805 us (+ alpha)
    assert abs(ring_allreduce_us(69_000_000, 8, 150.0, 0.0) - 805.0) < 1.0
    assert ring_allreduce_us(0, 8, 150.0, 15.0) == 15.0


def test_ddp_stream_mode(monkeypatch):
    from robotic_discovery_platform_amd.train.engine import NativeTrainer
    monkeypatch.delenv("RDP_DDP_STREAM", raising=False)
    assert NativeTrainer.ddp_stream_mode(1) == "side"
    assert NativeTrainer.ddp_stream_mode(8) in ("side", "dedicated")
    monkeypatch.setenv("RDP_DDP_STREAM", "dedicated")
    assert NativeTrainer.ddp_stream_mode(1) == "dedicated"
    monkeypatch.setenv("RDP_DDP_STREAM", "bogus")
    with pytest.raises(ValueError):
        NativeTrainer.ddp_stream_mode(2)
