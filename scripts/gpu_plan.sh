#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export RDP_NO_BUILD=1
timeout -k 10 400 python -u -m pytest tests/test_unet_native_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/plan_test.log 2>&1
rc=$?; tail -4 gpurun_out/plan_test.log; [ $rc -eq 0 ] || exit $rc
for b in 4 64; do
KNOB=RDP_PLAN_GRAPH VALS="0 1" BARGS="--batch $b" bash scripts/gpu_knob_ab2.sh || exit 1
done
timeout -k 10 200 python scripts/host_bound.py 4 64
