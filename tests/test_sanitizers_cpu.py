"""Host sanitizer builds of the native host code (SURVEY.md §5 "race detection / sanitizers").

``csrc/spline.cpp`` (the FITPACK-equivalent fit behind every served frame) is compiled with
AddressSanitizer + UndefinedBehaviorSanitizer and driven over arcs, noisy clouds, all k in 1..5,
minimum-size knot buffers and degenerate inputs (tests/native/spline_sanitize_main.cpp). GPU
sanitizers are not available on the MI355X pool; the device kernels are covered by the race
screens in test_race_screens_gpu.py instead.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
@pytest.mark.parametrize("san", ["address,undefined"])
def test_spline_host_sanitizers(tmp_path, san):
    exe = str(tmp_path / "spline_san")
    cmd = ["g++", "-std=c++17", "-O1", "-g", f"-fsanitize={san}", "-fno-sanitize-recover=all",
           "-fno-omit-frame-pointer", os.path.join(ROOT, "csrc", "spline.cpp"),
           os.path.join(ROOT, "tests", "native", "spline_sanitize_main.cpp"), "-o", exe]
    b = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    if b.returncode != 0 and "asan" in (b.stderr or "").lower():
        pytest.skip("sanitizer runtime not installed: " + b.stderr[-200:])
    assert b.returncode == 0, b.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout
