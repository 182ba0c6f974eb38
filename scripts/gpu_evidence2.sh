#!/bin/bash
# wgrad microbench + PMC with the halo kernel at its full split count, and the serving-frame kernel trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R"; mkdir -p gpurun_out/ev2
export RDP_NO_BUILD=1 PYTHONPATH=$R
timeout -k 10 240 python scripts/conv_microbench.py --batch 64 --variants 0,4 --wgrad --wgrad-blocks 512 --reps 5 --rounds 3 --out gpurun_out/ev2/micro_wgrad.json > gpurun_out/ev2/micro_wgrad.log 2>&1 || { tail -5 gpurun_out/ev2/micro_wgrad.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $line -d $R/gpurun_out/ev2/pmc_wgrad/set$i -o pmc --output-format csv -- python3 $R/scripts/conv_microbench.py --batch 64 --variants 0 --wgrad --wgrad-blocks 512 --reps 1 --rounds 1 > $R/gpurun_out/ev2/pmc_wgrad_set$i.log 2>&1 || { echo "wgrad set $i failed"; exit 1; }
done < $R/scripts/pmc_sets_r3.txt
echo pmc_ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ev2/prof_serve -o serve --output-format csv -- python3 -m robotic_discovery_platform_amd.serve.bench_serve --frames 200 --warmup 20 --train-steps 200 --e2e 0 --multi 0 > $R/gpurun_out/ev2/prof_serve.log 2>&1 || { tail -20 $R/gpurun_out/ev2/prof_serve.log; exit 1; }
echo prof_ok
