#!/bin/bash
# Serving A/B of one env knob incl. the e2e gRPC path: KNOB=NAME VALUES="a b" [ROUNDS=2] [E2E=1]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export RDP_NO_BUILD=1
for round in $(seq 1 ${ROUNDS:-2}); do
for v in $VALUES; do
  env "$KNOB=$v" timeout -k 10 300 python -m robotic_discovery_platform_amd.serve.bench_serve --frames ${FRAMES:-400} --warmup 40 --train-steps ${TRAIN_STEPS:-200} --e2e ${E2E:-1} > gpurun_out/sab_${v}_$round.json 2> gpurun_out/sab_${v}_$round.err || { tail -20 gpurun_out/sab_${v}_$round.err; exit 1; }
  echo "$KNOB=$v round$round $(python3 -c "import json;d=json.load(open('gpurun_out/sab_${v}_$round.json'));print({k:v for k,v in d.items() if ('p50' in k or 'fps' in k or 'p99' in k)})")"
done
done
