#!/bin/bash
# DDP on one GPU: the DDP / RCCL GPU tests, then the forced-DDP step (1-rank nccl) against the plain
# step at bs 4 and bs 64 (native RCCL issue; RDP_DDP_COMM=torch for the torch.distributed issue).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export RDP_NO_BUILD=1
timeout -k 10 500 python -u -m pytest tests/test_ddp_rccl_gpu.py tests/test_ddp_native_gpu.py tests/test_kernels_gpu.py \
  -k "ddp or rccl or bucket or adam" -x -v --timeout 300 --timeout-method thread > gpurun_out/ddp.log 2>&1 \
  || { tail -40 gpurun_out/ddp.log; exit 1; }
tail -16 gpurun_out/ddp.log
run() {  # label, env..., -- bench args
  local label=$1; shift
  env "$@" timeout -k 10 200 python bench.py --serve 0 --extras 0 ${ARGS} > gpurun_out/ddp_bench.json 2> gpurun_out/ddp_bench.err \
    || { tail -20 gpurun_out/ddp_bench.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/ddp_bench.json').read().splitlines()[-1]);print('$label',d['value'],d['ms_per_step'])"
}
for r in 1 2; do
  ARGS="--batch 4 --steps 200 --warmup 20" run "bs4 plain r$r" X=1
  ARGS="--batch 4 --steps 200 --warmup 20 --ddp-force 1" run "bs4 ddp-native r$r" X=1
done
ARGS="--batch 4 --steps 200 --warmup 20 --ddp-force 1" run "bs4 ddp-torch" RDP_DDP_COMM=torch
ARGS="--batch 4 --steps 200 --warmup 20 --ddp-force 1 --grad-comm bf16" run "bs4 ddp-native-bf16" X=1
ARGS="--batch 64 --steps 20 --warmup 5" run "bs64 plain" X=1
ARGS="--batch 64 --steps 20 --warmup 5 --ddp-force 1" run "bs64 ddp-native" X=1
