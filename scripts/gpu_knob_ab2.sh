#!/bin/bash
# Interleaved bench A/B of one env knob: KNOB=name VALS="a b" (bs 64 default step, no extras)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export RDP_NO_BUILD=1
for i in 1 2; do
  for v in $VALS; do
    env $KNOB=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --serve 0 --extras 0 ${BARGS} > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { tail -20 gpurun_out/ab_$v.err; exit 1; }
    echo "$KNOB=$v $(python -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print(d['value'], d['ms_per_step'])")"
  done
done
