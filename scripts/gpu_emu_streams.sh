#!/bin/bash
# Which issue stream at world > 1 -- and does the answer depend on which hardware queue the streams land on?
# side vs dedicated, with / without the self-check's probe stream created first (it shifts the round-robin
# stream -> hardware-queue assignment of every later stream); emulated n = 8, 150 GB/s, 16 CUs, no traffic.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export RDP_NO_BUILD=1
: > gpurun_out/emu_streams.txt
run() {
  local lab=$1 envs=$2 b=$3 st
  st=$([ $b = 4 ] && echo 150 || echo 20)
  env $envs timeout -k 10 200 python bench.py --ddp-force 1 --batch $b --steps $st --warmup 5 --serve 0 --extras 0 \
    > gpurun_out/emu.json 2> gpurun_out/emu.err || { tail -20 gpurun_out/emu.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/emu.json').read().splitlines()[-1]);print('$lab bs$b',d['value'],d['ms_per_step'])" | tee -a gpurun_out/emu_streams.txt
}
E="RDP_DDP_EMULATE=8:150:16:15:0"
for r in 1 2; do for b in 64 4; do
  run "side probe r$r" "$E RDP_DDP_STREAM=side" $b || exit 1
  run "dedicated probe r$r" "$E RDP_DDP_STREAM=dedicated" $b || exit 1
  run "side noprobe r$r" "$E RDP_DDP_STREAM=side RDP_COMM_SELFCHECK=0" $b || exit 1
  run "dedicated noprobe r$r" "$E RDP_DDP_STREAM=dedicated RDP_COMM_SELFCHECK=0" $b || exit 1
  run "dedicated probe 32cu-traffic r$r" "RDP_DDP_EMULATE=8:150:32:15:3 RDP_DDP_STREAM=dedicated" $b || exit 1
  run "side probe 32cu-traffic r$r" "RDP_DDP_EMULATE=8:150:32:15:3 RDP_DDP_STREAM=side" $b || exit 1
done; done
