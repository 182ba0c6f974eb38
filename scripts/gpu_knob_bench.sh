#!/bin/bash
# bench.py A/B of one env knob (in-tree build): KNOB=NAME VALUES="a b c" BATCHES="4 64", 2 rounds
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export RDP_NO_BUILD=1
for round in 1 2; do
for v in $VALUES; do
  for b in ${BATCHES:-64}; do
    env "$KNOB=$v" timeout -k 10 300 python bench.py --batch $b --steps ${STEPS:-20} --warmup 5 --serve 0 --extras 0 > gpurun_out/kb_${v}_b${b}_$round.json 2> gpurun_out/kb_${v}_b${b}_$round.err || { tail -20 gpurun_out/kb_${v}_b${b}_$round.err; exit 1; }
    echo "$KNOB=$v b$b round$round $(python3 -c "import json;d=json.load(open('gpurun_out/kb_${v}_b${b}_$round.json'));print(d['value'], d['ms_per_step'])")"
  done
done
done
