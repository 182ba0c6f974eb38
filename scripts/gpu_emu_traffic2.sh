#!/bin/bash
# Round 6: emulated n = 8 collectives with / without their HBM traffic (RDP_DDP_EMULATE 5th field), side vs
# dedicated issue stream, fp32 vs bf16 buckets, bs 64 and bs 4, 2 interleaved rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export RDP_NO_BUILD=1
: > gpurun_out/emu_traffic2.txt
run() {  # label, env, args
  local lab=$1 envs=$2 args=$3 b=$4 st
  st=$([ $b = 4 ] && echo 150 || echo 20)
  env $envs timeout -k 10 200 python bench.py --ddp-force 1 --batch $b --steps $st --warmup 5 --serve 0 --extras 0 $args \
    > gpurun_out/emu.json 2> gpurun_out/emu.err || { tail -20 gpurun_out/emu.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/emu.json').read().splitlines()[-1]);print('$lab bs$b',d['value'],d['ms_per_step'])" | tee -a gpurun_out/emu_traffic2.txt
}
for r in 1 2; do for b in 64 4; do
  run "spin-side-fp32 r$r" "RDP_DDP_EMULATE=8:150:16:15:0" "" $b || exit 1
  run "spin-dedicated-fp32 r$r" "RDP_DDP_EMULATE=8:150:16:15:0 RDP_DDP_STREAM=dedicated" "" $b || exit 1
  run "traffic-side-fp32 r$r" "RDP_DDP_EMULATE=8:150:16:15:3" "" $b || exit 1
  run "traffic-dedicated-fp32 r$r" "RDP_DDP_EMULATE=8:150:16:15:3 RDP_DDP_STREAM=dedicated" "" $b || exit 1
  run "traffic-dedicated-bf16 r$r" "RDP_DDP_EMULATE=8:150:16:15:3 RDP_DDP_STREAM=dedicated" "--grad-comm bf16" $b || exit 1
done; done
