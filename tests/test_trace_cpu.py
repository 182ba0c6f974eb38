"""roctx markers: no-ops when disabled, balanced push/pop when the library is present."""
from robotic_discovery_platform_amd.utils import trace


def test_trace_disabled_is_noop():
    trace.enable(False)
    with trace.range("x"):
        with trace.range("y"):
            pass
    trace.mark("m")


def test_trace_enabled_if_library_present():
    ok = trace.enable(True)
    try:
        with trace.range("outer"):
            trace.mark("inside")
        assert trace.enabled() == ok
    finally:
        trace.enable(False)
