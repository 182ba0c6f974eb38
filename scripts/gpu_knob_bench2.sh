#!/bin/bash
# bench.py A/B of one env knob, interleaved over values, bs4 with 200 timed steps and bs64 with 30:
# KNOB=NAME VALUES="a b c" [BATCHES="4 64"] [ROUNDS=2]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export RDP_NO_BUILD=1
for round in $(seq 1 ${ROUNDS:-2}); do
for b in ${BATCHES:-4 64}; do
  steps=30; [ "$b" -le 8 ] && steps=200
  for v in $VALUES; do
    env "$KNOB=$v" timeout -k 10 300 python bench.py --batch $b --steps $steps --warmup 10 --serve 0 --extras 0 > gpurun_out/kb_${v}_b${b}_$round.json 2> gpurun_out/kb_${v}_b${b}_$round.err || { tail -20 gpurun_out/kb_${v}_b${b}_$round.err; exit 1; }
    echo "$KNOB=$v b$b round$round $(python3 -c "import json;d=json.load(open('gpurun_out/kb_${v}_b${b}_$round.json'));print(d['value'], d['ms_per_step'])")"
  done
done
done
