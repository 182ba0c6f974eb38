#!/bin/bash
# Env-knob sweep of the bs-64 training step (each config twice, interleaved).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export RDP_NO_BUILD=1
B=${B:-64}
for round in 1 2; do
  i=0
  while IFS= read -r cfg; do
    [ -z "$cfg" ] && continue
    i=$((i+1))
    env $cfg timeout -k 10 200 python bench.py --batch $B --steps ${STEPS:-15} --warmup 4 --serve 0 --extras 0 ${BENCH_ARGS} > gpurun_out/sw_$i.json 2> gpurun_out/sw_$i.err || { echo "FAIL $cfg"; tail -5 gpurun_out/sw_$i.err; exit 1; }
    echo "r$round [$cfg] $(python3 -c "import json;d=json.load(open('gpurun_out/sw_$i.json'));print(d['value'], d['ms_per_step'])")"
  done < ${CFGS:-scripts/sweep_cfgs.txt}
done
