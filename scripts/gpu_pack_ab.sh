#!/bin/bash
# single-instruction bf16 pair pack: kernel tests, ring / ping-pong kernel times, step bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/pack
export RDP_NO_BUILD=1
timeout -k 10 700 python -u -m pytest tests/test_kernels_gpu.py tests/test_unet_native_gpu.py -x -q --timeout 240 \
  --timeout-method thread > gpurun_out/pack/tests.log 2>&1
rc=$?; tail -3 gpurun_out/pack/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/conv_microbench.py --batch 64 --shapes 0 --variants 0,9,10 --rounds 5 --reps 10 \
  > gpurun_out/pack/fwd.jsonl 2>&1 || exit 1
timeout -k 10 200 python -u scripts/conv_microbench.py --batch 64 --shapes 3,4,9 --variants 0 --rounds 5 --reps 10 \
  >> gpurun_out/pack/fwd.jsonl 2>&1 || exit 1
timeout -k 10 200 python -u scripts/conv_microbench.py --batch 4 --shapes 0 --variants 0,9,10 --rounds 5 --reps 20 \
  >> gpurun_out/pack/fwd.jsonl 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/pack/fwd.jsonl
run() {  # batch steps tag
  local b=$1 st=$2 tag=$3
  timeout -k 10 300 python bench.py --batch $b --steps $st --warmup 5 --serve 0 --extras 0 \
    > gpurun_out/pack/b.json 2>> gpurun_out/pack/bench.err || exit 1
  echo "b$b $tag $(python -c "import json;d=json.load(open('gpurun_out/pack/b.json'));print(d['value'],d['ms_per_step'])")"
}
for r in 1 2; do run 64 25 "r$r"; done
for r in 1 2; do run 4 60 "r$r"; done
