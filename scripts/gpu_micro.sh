#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export RDP_NO_BUILD=1
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python scripts/conv_microbench.py ${MB_ARGS} --out gpurun_out/micro.json 2>&1 | tee gpurun_out/micro.log || exit 1
timeout -k 10 300 python bench.py --batch 32 --steps 20 --warmup 5 > gpurun_out/native_b32.json 2>gpurun_out/native_b32.err || { tail gpurun_out/native_b32.err; exit 1; }
cat gpurun_out/native_b32.json | cut -c1-200
