#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export RDP_NO_BUILD=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_unet_native_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/first_test.log 2>&1
rc=$?; tail -4 gpurun_out/first_test.log; [ $rc -eq 0 ] || exit $rc
for b in 64 4; do
KNOB=RDP_CONV_FIRST VALS="0 1" BARGS="--batch $b" bash scripts/gpu_knob_ab2.sh || exit 1
done
