#!/bin/bash
# Side-stream fork grouping (RDP_FORK_GROUP): native training / DDP GPU tests, interleaved step A/B at bs 4,
# conv microbench of the split-K ping-pong on the dgrad shapes.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R"; mkdir -p gpurun_out/fork
export RDP_NO_BUILD=1
timeout -k 10 600 python -u -m pytest tests/test_unet_native_gpu.py tests/test_ddp_native_gpu.py tests/test_ddp_rccl_gpu.py \
  tests/test_train_serve_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/fork/tests.log 2>&1
rc=$?; tail -4 gpurun_out/fork/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in 1 2 3; do
    RDP_FORK_GROUP=$v timeout -k 10 300 python bench.py --batch 4 --steps 60 --warmup 8 --serve 0 --extras 0 \
      > gpurun_out/fork/b4_$v.json 2>> gpurun_out/fork/bench.err || exit 1
    echo "b4 fork=$v round $r $(python -c "import json;d=json.load(open('gpurun_out/fork/b4_$v.json'));print(d['value'],d['ms_per_step'])")"
  done
done
timeout -k 10 300 python -u scripts/conv_microbench.py --batch 4 --variants 2,7,0 --ws 1 --reps 20 --rounds 5 \
  --shapes 18,19,20,13,6 > gpurun_out/fork/micro.jsonl 2>&1 || { tail -5 gpurun_out/fork/micro.jsonl; exit 1; }
cat gpurun_out/fork/micro.jsonl
