#!/bin/bash
# serving GPU tests, then the serving bench (engine + e2e) with the pinned-staging A/B (RDP_STAGE_TORCH 0 / 1)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export RDP_NO_BUILD=1
timeout -k 10 400 python -u -m pytest tests/test_serve_gpu.py tests/test_train_serve_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_serve.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_serve.log; [ $rc -eq 0 ] || exit $rc
KNOB=RDP_STAGE_TORCH VALUES="0 1" ROUNDS=2 bash scripts/gpu_serve_ab2.sh
