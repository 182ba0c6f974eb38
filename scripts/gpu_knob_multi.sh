#!/bin/bash
# Several env-knob A/Bs at bs64 (30 timed steps), each value interleaved with the default over 2 rounds.
# KNOBS="NAME=v1,v2 NAME2=v1" ; the default run ("base") is repeated in every round.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export RDP_NO_BUILD=1
b=${BATCH:-64}
for kv in $KNOBS; do
  k=${kv%%=*}; vals=${kv#*=}
  for round in 1 2; do
    for v in base ${vals//,/ }; do
      if [ "$v" = base ]; then envs=""; else envs="$k=$v"; fi
      env $envs timeout -k 10 300 python bench.py --batch $b --steps ${STEPS:-30} --warmup 8 --serve 0 --extras 0 > gpurun_out/km.json 2> gpurun_out/km.err || { tail -20 gpurun_out/km.err; exit 1; }
      echo "$k=$v b$b round$round $(python3 -c "import json;d=json.load(open('gpurun_out/km.json'));print(d['value'], d['ms_per_step'])")"
    done
  done
done
