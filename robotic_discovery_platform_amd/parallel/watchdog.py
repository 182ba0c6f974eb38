"""Host watchdog for natively issued RCCL collectives.

The DDP bucket all-reduces are enqueued with ``ncclAllReduce`` straight onto the executor's HIP stream
(``csrc/bindings.cpp`` comm_all_reduce, ``parallel/ddp.py``). That skips ProcessGroupNCCL's work
objects, so c10d's own watchdog and its timeout never cover them: a dead or stalled peer would block
the stream -- and with it the next host synchronisation -- forever, with no error.

:class:`CommWatchdog` closes that gap. Each training step that issued native collectives ``arm``s it
with an event recorded after the step's work (its completion means every collective of the step has
finished). A daemon thread polls, every ``period`` seconds while anything is armed:

  * the communicator's asynchronous error (``ncclCommGetAsyncError``): non-zero -> failure;
  * the oldest armed event: still incomplete ``timeout`` seconds after it was armed -> failure.

On failure it aborts the communicator (``ncclCommAbort``, which releases the kernels waiting on the
peer), writes one rank-tagged line to stderr and ends the process with a non-zero status, so the
launcher (torchrun) tears the job down and ``train_model(resume="auto")`` can relaunch it from the last
checkpoint -- the same contract as the process-group timeout (``utils/launch.py`` dist_timeout).
``RDP_DDP_COMM=torch`` issues through torch.distributed instead, where c10d's timeouts apply.

Everything device-specific is injected (``poll``, ``abort``, events with ``query()``), so the failure
paths are tested on CPU with fakes (``tests/test_watchdog_cpu.py``).
"""
from __future__ import annotations

import collections
import os
import sys
import threading
import time
from typing import Callable, Deque, Optional, Tuple

EXIT_CODE = 75  # distinct from a crash (1) / injected fault (17) in merged launcher logs

_LIVE: "list[CommWatchdog]" = []


def close_all() -> None:
    """Stop every watchdog of this process: call before destroying the process groups whose
    communicators they poll (utils/launch.py shutdown_distributed, bench.py)."""
    while _LIVE:
        _LIVE.pop().close()


def _default_fail(msg: str) -> None:
    sys.stderr.write(msg + "\n")
    sys.stderr.flush()
    os._exit(EXIT_CODE)


class CommWatchdog:
    def __init__(self, poll: Callable[[], Tuple[int, str]], abort: Optional[Callable[[], object]] = None,
                 timeout: Optional[float] = None, period: float = 1.0, rank: Optional[int] = None,
                 on_fail: Optional[Callable[[str], None]] = None, max_armed: int = 64):
        if timeout is None:
            timeout = float(os.environ.get("RDP_DIST_TIMEOUT_S", "600"))
        self.poll, self.abort = poll, abort
        self.timeout, self.period = float(timeout), float(period)
        self.rank = int(os.environ.get("RANK", "0")) if rank is None else int(rank)
        self.on_fail = on_fail or _default_fail
        self.max_armed = max_armed
        self._armed: Deque[Tuple[float, object]] = collections.deque()
        self._lock = threading.Lock()
        self._wake = threading.Event()
        self._stop = threading.Event()
        self.failed: Optional[str] = None
        self._thread = threading.Thread(target=self._run, name="rdp-comm-watchdog", daemon=True)
        self._thread.start()
        _LIVE.append(self)

    def arm(self, event) -> None:
        """Watch ``event`` (anything with ``query() -> bool``: done). Called once per step from the
        training thread; bounded (the oldest entries are the ones that matter)."""
        with self._lock:
            self._armed.append((time.monotonic(), event))
            while len(self._armed) > self.max_armed:  # the host ran far ahead: keep the oldest and newest
                del self._armed[1]
        self._wake.set()

    def pending(self) -> int:
        with self._lock:
            return len(self._armed)

    def close(self) -> None:
        self._stop.set()
        self._wake.set()
        with self._lock:  # a poll in progress finishes before the caller may free the communicator
            pass
        self._thread.join(timeout=5.0)
        if self in _LIVE:
            _LIVE.remove(self)

    def _fail(self, why: str) -> None:
        self.failed = why
        msg = f"[rank {self.rank}] RDP comm watchdog: {why}"
        if self.abort is not None:
            try:
                self.abort()
            except Exception as e:  # the process is ending anyway
                msg += f" (abort failed: {type(e).__name__}: {e})"
        self.on_fail(msg)

    def check_once(self) -> bool:
        """One poll; returns False once a failure was reported."""
        if self.failed is not None:
            return False
        with self._lock:
            if self._stop.is_set():
                return True
            while self._armed and self._armed[0][1].query():
                self._armed.popleft()
            oldest = self._armed[0] if self._armed else None
            if oldest is None:
                return True
            code, text = self.poll()  # under the lock: close() waits for a poll in progress
        if code:
            self._fail(f"collective failed with RCCL error {code}: {text}")
            return False
        age = time.monotonic() - oldest[0]
        if age > self.timeout:
            self._fail(f"collectives of a step still incomplete after {age:.0f} s (timeout {self.timeout:.0f} s)")
            return False
        return True

    def _run(self) -> None:
        while not self._stop.is_set():
            if not self.pending():
                self._wake.wait()
                self._wake.clear()
                continue
            if not self.check_once():
                return
            self._stop.wait(self.period)
