#!/bin/bash
# Kernel traces of one bench configuration under two environment settings (A/B), summarised per step:
# PROF_ENV="E=a E=b" PROF_ARGS="--batch 4 --steps 20 --warmup 5" bash scripts/gpu_prof_ab.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R"; mkdir -p gpurun_out/pab
export RDP_NO_BUILD=1 PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
i=0
for e in $PROF_ENV; do
  i=$((i+1))
  env ${e//,/ } timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pab/p$i -o p --output-format csv -- python3 $R/bench.py $PROF_ARGS --serve 0 --extras 0 > $R/gpurun_out/pab/p$i.log 2>&1 || { tail -20 $R/gpurun_out/pab/p$i.log; exit 1; }
  f=$(find $R/gpurun_out/pab/p$i -name '*kernel_trace.csv' | head -1)
  python3 $R/scripts/step_profile_md.py "$f" "$e $PROF_ARGS" --sequence > $R/gpurun_out/pab/p$i.md || exit 1
  rm -f "$f"
  head -12 $R/gpurun_out/pab/p$i.md | tail -6
done
