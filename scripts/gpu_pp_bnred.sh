#!/bin/bash
# ping-pong dgrad + BN-backward reduction: kernel + model tests, then the bench A/B (RDP_DGRAD_PP_BNRED 0 / 1).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export RDP_NO_BUILD=1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_unet_native_gpu.py -x -q --timeout 200 --timeout-method thread -k "pp_bnred or first or unet or native or bitwise or plan" > gpurun_out/pytest_ppbnred.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_ppbnred.log; [ $rc -eq 0 ] || exit $rc
KNOB=RDP_DGRAD_PP_BNRED VALUES="0 1" ROUNDS=3 bash scripts/gpu_knob_bench2.sh
