#!/bin/bash
# Serving-engine A/B of one env knob in the in-tree build: KNOB=NAME, A=value, B=value (2 rounds).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export RDP_NO_BUILD=1
for round in 1 2; do
for v in "$A" "$B"; do
  env "$KNOB=$v" timeout -k 10 300 python -m robotic_discovery_platform_amd.serve.bench_serve --frames ${FRAMES:-400} --warmup 40 --train-steps ${TRAIN_STEPS:-200} --e2e 0 > gpurun_out/kab_${v}_$round.json 2> gpurun_out/kab_${v}_$round.err || { tail -20 gpurun_out/kab_${v}_$round.err; exit 1; }
  echo "$KNOB=$v round$round $(python3 -c "import json;d=json.load(open('gpurun_out/kab_${v}_$round.json'));print({k:v for k,v in d.items() if 'p50' in k or 'fps' in k})")"
done
done
