#!/bin/bash
# BN finalize channels-per-block A/B (RDP_FIN_CPB 64 / 16): BN / model tests under 16, then the bench at bs4 and bs64
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export RDP_NO_BUILD=1
RDP_FIN_CPB=16 timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_unet_native_gpu.py -x -q --timeout 200 --timeout-method thread -k "bn or unet or native" > gpurun_out/pytest_fin.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_fin.log; [ $rc -eq 0 ] || exit $rc
KNOB=RDP_FIN_CPB VALUES="64 16" ROUNDS=2 bash scripts/gpu_knob_bench2.sh
