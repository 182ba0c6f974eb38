#!/bin/bash
# pp dgrad + BN-backward reduction A/B: off / on for both tile widths / on for the 256x128 form only
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export RDP_NO_BUILD=1
for round in 1 2 3; do
  for cfg in "RDP_DGRAD_PP_BNRED=0" "RDP_DGRAD_PP_BNRED=1" "RDP_DGRAD_PP_BNRED=1 RDP_PP_BNRED_WIDTH=128"; do
    env $cfg timeout -k 10 300 python bench.py --batch 64 --steps 30 --warmup 8 --serve 0 --extras 0 > gpurun_out/pb.json 2> gpurun_out/pb.err || { tail -20 gpurun_out/pb.err; exit 1; }
    echo "$cfg round$round $(python3 -c "import json;d=json.load(open('gpurun_out/pb.json'));print(d['value'], d['ms_per_step'])")"
  done
done
