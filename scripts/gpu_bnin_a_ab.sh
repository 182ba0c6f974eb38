#!/bin/bash
# BNIN forward that also stores the activation (RDP_BNIN_WRITE_A): GPU tests and step A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/bnina
export RDP_NO_BUILD=1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_unet_native_gpu.py -x -q --timeout 240 \
  --timeout-method thread -k "bnin or native or plan or wprep" > gpurun_out/bnina/tests.log 2>&1
rc=$?; tail -3 gpurun_out/bnina/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/conv_microbench.py --batch 64 --shapes 0 --variants 0,9,10 --rounds 5 --reps 10 \
  > gpurun_out/bnina/fwd.jsonl 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/bnina/fwd.jsonl
run() {  # batch steps tag env...
  local b=$1 st=$2 tag=$3; shift 3
  env "$@" timeout -k 10 300 python bench.py --batch $b --steps $st --warmup 5 --serve 0 --extras 0 \
    > gpurun_out/bnina/b.json 2>> gpurun_out/bnina/bench.err || exit 1
  echo "b$b $tag $(python -c "import json;d=json.load(open('gpurun_out/bnina/b.json'));print(d['value'],d['ms_per_step'])")"
}
for r in 1 2 3; do
  run 64 25 "wa=0 r$r" RDP_BNIN_WRITE_A=0
  run 64 25 "wa=1 r$r" RDP_BNIN_WRITE_A=1
done
for r in 1 2; do
  run 4 60 "wa=0 r$r" RDP_BNIN_WRITE_A=0
  run 4 60 "wa=1 r$r" RDP_BNIN_WRITE_A=1
done
