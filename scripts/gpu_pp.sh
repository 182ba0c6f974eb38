#!/bin/bash
# Ping-pong conv kernel: bitwise tests + A/B microbench vs the 128x128 kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export RDP_NO_BUILD=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "pingpong or conv_fwd_and_stats or pipeline_depth" > gpurun_out/pp_test.log 2>&1
rc=$?; tail -15 gpurun_out/pp_test.log; [ $rc -eq 0 ] || exit $rc
for b in ${BATCHES:-64}; do
  timeout -k 10 300 python -u scripts/conv_microbench.py --batch $b --shapes 3,4,6 --variants 0,4,7,9,10 --rounds 5 > gpurun_out/pp_mb_a_$b.log 2>&1 || { tail -20 gpurun_out/pp_mb_a_$b.log; exit 1; }
  tail -6 gpurun_out/pp_mb_a_$b.log
  timeout -k 10 300 python -u scripts/conv_microbench.py --batch $b --shapes 1,2,7 --variants 0,5,8 --rounds 5 > gpurun_out/pp_mb_b_$b.log 2>&1 || { tail -20 gpurun_out/pp_mb_b_$b.log; exit 1; }
  tail -5 gpurun_out/pp_mb_b_$b.log
done
if [ -n "$BENCHAB" ]; then
  for i in 1 2; do
    for pp in 0 1; do
      RDP_CONV_PP=$pp timeout -k 10 300 python bench.py --steps 20 --warmup 5 --serve 0 --extras 0 > gpurun_out/pp_bench_$pp.json 2> gpurun_out/pp_bench_$pp.err || { tail -20 gpurun_out/pp_bench_$pp.err; exit 1; }
      echo "pp=$pp $(python -c "import json;d=json.load(open('gpurun_out/pp_bench_$pp.json'));print(d['value'], d['ms_per_step'])")"
    done
  done
fi
