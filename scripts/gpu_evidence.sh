#!/bin/bash
# Round-3 evidence refresh (one GPU call): conv microbench (fwd auto dispatch + wgrad), PMC counters for
# the conv / wgrad kernels (microbench) and the first layer's fused wgrad (training step), kernel traces
# of the bs-64 and bs-4 training steps and of the serving frames. Each step under its own time limit.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R"; mkdir -p gpurun_out/ev
export RDP_NO_BUILD=1 PYTHONPATH=$R
timeout -k 10 240 python scripts/conv_microbench.py --batch 64 --variants 0 --reps 10 --rounds 3 --out gpurun_out/ev/micro_fwd.json > gpurun_out/ev/micro_fwd.log 2>&1 || { tail -5 gpurun_out/ev/micro_fwd.log; exit 1; }
timeout -k 10 240 python scripts/conv_microbench.py --batch 64 --variants 0,4 --wgrad --wgrad-blocks 512 --reps 5 --rounds 3 --out gpurun_out/ev/micro_wgrad.json > gpurun_out/ev/micro_wgrad.log 2>&1 || { tail -5 gpurun_out/ev/micro_wgrad.log; exit 1; }
echo micro_ok
cd /tmp && export TMPDIR=/tmp
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $line -d $R/gpurun_out/ev/pmc_fwd/set$i -o pmc --output-format csv -- python3 $R/scripts/conv_microbench.py --batch 64 --variants 0 --reps 1 --rounds 1 > $R/gpurun_out/ev/pmc_fwd_set$i.log 2>&1 || { echo "fwd set $i failed"; exit 1; }
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $line -d $R/gpurun_out/ev/pmc_wgrad/set$i -o pmc --output-format csv -- python3 $R/scripts/conv_microbench.py --batch 64 --variants 0 --wgrad --wgrad-blocks 512 --reps 1 --rounds 1 > $R/gpurun_out/ev/pmc_wgrad_set$i.log 2>&1 || { echo "wgrad set $i failed"; exit 1; }
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $line -d $R/gpurun_out/ev/pmc_step/set$i -o pmc --output-format csv -- python3 $R/bench.py --batch 64 --steps 2 --warmup 1 --serve 0 --extras 0 > $R/gpurun_out/ev/pmc_step_set$i.log 2>&1 || { echo "step set $i failed"; exit 1; }
done < $R/scripts/pmc_sets_r3.txt
echo pmc_ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ev/prof_train -o train --output-format csv -- python3 $R/bench.py --batch 64 --steps 4 --warmup 3 --serve 0 --extras 0 > $R/gpurun_out/ev/prof_train.log 2>&1 || { tail -20 $R/gpurun_out/ev/prof_train.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ev/prof_bs4 -o bs4 --output-format csv -- python3 $R/bench.py --batch 4 --steps 20 --warmup 5 --serve 0 --extras 0 > $R/gpurun_out/ev/prof_bs4.log 2>&1 || { tail -20 $R/gpurun_out/ev/prof_bs4.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ev/prof_serve -o serve --output-format csv -- python3 -m robotic_discovery_platform_amd.serve.bench_serve --frames 200 --warmup 20 --train-steps 200 --e2e 0 > $R/gpurun_out/ev/prof_serve.log 2>&1 || { tail -20 $R/gpurun_out/ev/prof_serve.log; exit 1; }
echo prof_ok
