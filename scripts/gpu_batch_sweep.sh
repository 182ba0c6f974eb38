#!/bin/bash
# per-GPU batch sweep of the default training step (2 interleaved rounds)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export RDP_NO_BUILD=1
for round in 1 2; do
for b in ${BATCHES:-48 64 96 128}; do
  timeout -k 10 300 python bench.py --batch $b --steps 20 --warmup 5 --serve 0 --extras 0 > gpurun_out/bs_${b}_$round.json 2> gpurun_out/bs_${b}_$round.err || { tail -20 gpurun_out/bs_${b}_$round.err; exit 1; }
  echo "b$b round$round $(python3 -c "import json;d=json.load(open('gpurun_out/bs_${b}_$round.json'));print(d['value'], d['ms_per_step'])")"
done
done
