#!/bin/bash
# Staggered halo wgrad: bitwise tests, microbench (5 = halo, 7 = staggered halo), bench A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export RDP_NO_BUILD=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "wgrad" > gpurun_out/wg_test.log 2>&1
rc=$?; tail -8 gpurun_out/wg_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/conv_microbench.py --wgrad --batch 64 --shapes 1,2,3,7,8 --variants 5,7 --rounds 5 --wgrad-blocks 512 > gpurun_out/wg_mb.log 2>&1 || { tail -20 gpurun_out/wg_mb.log; exit 1; }
tail -5 gpurun_out/wg_mb.log
for i in 1 2; do
  for st in 0 1; do
    RDP_WGRAD_STAG=$st timeout -k 10 300 python bench.py --steps 20 --warmup 5 --serve 0 --extras 0 > gpurun_out/wg_bench_$st.json 2> gpurun_out/wg_bench_$st.err || { tail -20 gpurun_out/wg_bench_$st.err; exit 1; }
    echo "stag=$st $(python -c "import json;d=json.load(open('gpurun_out/wg_bench_$st.json'));print(d['value'], d['ms_per_step'])")"
  done
done
