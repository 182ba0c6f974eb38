#!/bin/bash
# rocprofv3 kernel-time profiles of (a) the native training step and (b) the per-frame serving
# engine; summaries are written under gpurun_out/ and copied into profiles/ by scripts/profile_summary.py.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export RDP_NO_BUILD=1
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
[ -n "$SKIP_TRAIN" ] || RDP_WGRAD_OVERLAP=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_train -o train --output-format csv -- \
  python3 $R/bench.py --impl native --batch ${BATCH:-32} --steps 3 --warmup 2 --graph 0 --serve 0 > $R/gpurun_out/prof_train.log 2>&1 || { echo train_prof_failed; tail -20 $R/gpurun_out/prof_train.log; exit 1; }
echo train_prof_ok
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_serve -o serve --output-format csv -- \
  python3 -m robotic_discovery_platform_amd.serve.bench_serve --frames 50 --warmup 10 --train-steps 20 > $R/gpurun_out/prof_serve.log 2>&1 || { echo serve_prof_failed; tail -20 $R/gpurun_out/prof_serve.log; exit 1; }
echo serve_prof_ok
cd $R
timeout -k 10 300 python3 scripts/conv_microbench.py --variants 0,1,128 --rounds 3 > gpurun_out/micro_fwd.log 2>&1 || { echo micro_failed; exit 1; }
timeout -k 10 300 python3 scripts/conv_microbench.py --wgrad --variants 0,4 --rounds 3 > gpurun_out/micro_wgrad.log 2>&1 || { echo micro_failed; exit 1; }
cd $R && python3 scripts/profile_summary.py
