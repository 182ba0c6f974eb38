#!/bin/bash
# Split-K ping-pong conv: GPU tests, bs-4 layer microbench (igemm 128x128 split vs ping-pong split) and
# interleaved step A/B (RDP_PP_SPLIT=0 / 1) at the reference batch and at bs 64.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export RDP_NO_BUILD=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "pingpong or splitk or tiles_and_split" > gpurun_out/pp_tests.log 2>&1
rc=$?; tail -5 gpurun_out/pp_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/conv_microbench.py --batch 4 --variants 2,7,8,0 --ws 1 --reps 20 --rounds 5 \
  --shapes 3,4,5,6,7,12,13,14,15,16 > gpurun_out/pp_micro_b4.jsonl 2>&1 || { tail -5 gpurun_out/pp_micro_b4.jsonl; exit 1; }
cat gpurun_out/pp_micro_b4.jsonl
for r in 1 2; do
  for v in 0 1; do
    RDP_PP_SPLIT=$v timeout -k 10 200 python bench.py --batch 4 --steps 50 --warmup 10 --serve 0 --extras 0 \
      > gpurun_out/pp_b4_$v.json 2>> gpurun_out/pp_bench.err || exit 1
    echo "b4 split=$v round $r $(python -c "import json;d=json.load(open('gpurun_out/pp_b4_$v.json'));print(d['value'],d['ms_per_step'])")"
  done
done
for v in 0 1; do
  RDP_PP_SPLIT=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --serve 0 --extras 0 \
    > gpurun_out/pp_b64_$v.json 2>> gpurun_out/pp_bench.err || exit 1
  echo "b64 split=$v $(python -c "import json;d=json.load(open('gpurun_out/pp_b64_$v.json'));print(d['value'],d['ms_per_step'])")"
done
