#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export RDP_NO_BUILD=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "pingpong" > gpurun_out/pp_test.log 2>&1
rc=$?; tail -5 gpurun_out/pp_test.log; [ $rc -eq 0 ] || exit $rc
# 64-cout shapes: 10 = 256^2 64+64->64 (up4.0), 8 = 128^2 128+128->64, 9 = 256^2 64->64, 0 = 256^2 64->64
timeout -k 10 300 python -u scripts/conv_microbench.py --batch 64 --shapes 9,8,10 --variants 0,11,12 --rounds 5 > gpurun_out/pp64_mb.log 2>&1 || { tail -20 gpurun_out/pp64_mb.log; exit 1; }
tail -3 gpurun_out/pp64_mb.log
