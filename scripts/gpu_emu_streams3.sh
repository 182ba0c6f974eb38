#!/bin/bash
# Stream placement by probe (models.unet.concurrent_stream): dedicated collective stream with / without the
# self-check's probe stream, side stream, and the plain 1-GPU bench (no DDP) for regressions.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export RDP_NO_BUILD=1
timeout -k 10 600 python -u -m pytest tests/test_ddp_rccl_gpu.py tests/test_unet_native_gpu.py tests/test_bench_dist_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/streams_tests.log 2>&1 || { tail -30 gpurun_out/streams_tests.log; exit 1; }
tail -2 gpurun_out/streams_tests.log
: > gpurun_out/emu_streams3.txt
run() {
  local lab=$1 envs=$2 b=$3 st
  st=$([ "$b" = 4 ] && echo 150 || echo 20)
  env $envs timeout -k 10 200 python bench.py --batch $b --steps $st --warmup 5 --serve 0 --extras 0 $ARGS \
    > gpurun_out/emu.json 2> gpurun_out/emu.err || { tail -20 gpurun_out/emu.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/emu.json').read().splitlines()[-1]);print('$lab bs$b',d['value'],d['ms_per_step'],d['config'].get('ddp_stream'))" | tee -a gpurun_out/emu_streams3.txt
}
E="RDP_DDP_EMULATE=8:150:16:15:0"
for r in 1 2; do for b in 64 4; do
  ARGS="" run "plain (no DDP) r$r" "X=1" $b || exit 1
  ARGS="" run "plain, unprobed side stream r$r" "RDP_STREAM_PROBE=0" $b || exit 1
  ARGS="--ddp-force 1" run "default (dedicated) probe r$r" "$E" $b || exit 1
  ARGS="--ddp-force 1" run "default (dedicated) noprobe r$r" "$E RDP_COMM_SELFCHECK=0" $b || exit 1
  ARGS="--ddp-force 1" run "side r$r" "$E RDP_DDP_STREAM=side" $b || exit 1
done; done
