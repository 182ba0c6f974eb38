#!/bin/bash
# BN-on-input transform with the per-lane coefficients read once per stage: tests, kernel time, step bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/bninc
export RDP_NO_BUILD=1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_unet_native_gpu.py -x -q --timeout 240 \
  --timeout-method thread -k "bnin or native or plan" > gpurun_out/bninc/tests.log 2>&1
rc=$?; tail -2 gpurun_out/bninc/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/conv_microbench.py --batch 64 --shapes 0 --variants 0,9,10 --rounds 5 --reps 10 \
  > gpurun_out/bninc/fwd.jsonl 2>&1 || exit 1
timeout -k 10 200 python -u scripts/conv_microbench.py --batch 4 --shapes 0 --variants 0,9,10 --rounds 5 --reps 20 \
  >> gpurun_out/bninc/fwd.jsonl 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/bninc/fwd.jsonl
