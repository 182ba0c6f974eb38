#!/bin/bash
# The dedicated collective stream at high priority (its own hardware queues) vs normal priority, with / without
# the self-check's probe stream shifting the queue assignment; side stream for reference. Emulated n = 8, 150 GB/s.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export RDP_NO_BUILD=1
: > gpurun_out/emu_streams2.txt
run() {
  local lab=$1 envs=$2 b=$3 st
  st=$([ $b = 4 ] && echo 150 || echo 20)
  env $envs timeout -k 10 200 python bench.py --ddp-force 1 --batch $b --steps $st --warmup 5 --serve 0 --extras 0 \
    > gpurun_out/emu.json 2> gpurun_out/emu.err || { tail -20 gpurun_out/emu.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/emu.json').read().splitlines()[-1]);print('$lab bs$b',d['value'],d['ms_per_step'])" | tee -a gpurun_out/emu_streams2.txt
}
E="RDP_DDP_EMULATE=8:150:16:15:0"
for r in 1 2; do for b in 64 4; do
  run "side probe r$r" "$E RDP_DDP_STREAM=side" $b || exit 1
  run "dedicated-hi probe r$r" "$E RDP_DDP_STREAM=dedicated" $b || exit 1
  run "dedicated-hi noprobe r$r" "$E RDP_DDP_STREAM=dedicated RDP_COMM_SELFCHECK=0" $b || exit 1
  run "dedicated-lo noprobe r$r" "$E RDP_DDP_STREAM=dedicated RDP_COMM_SELFCHECK=0 RDP_DDP_COMM_PRIORITY=0" $b || exit 1
  run "dedicated-hi probe 300/32 r$r" "RDP_DDP_EMULATE=8:300:32:15:0 RDP_DDP_STREAM=dedicated" $b || exit 1
  run "side probe 300/32 r$r" "RDP_DDP_EMULATE=8:300:32:15:0 RDP_DDP_STREAM=side" $b || exit 1
  run "dedicated-hi probe bf16 r$r" "$E RDP_DDP_STREAM=dedicated" "$b --grad-comm bf16" || exit 1
done; done
