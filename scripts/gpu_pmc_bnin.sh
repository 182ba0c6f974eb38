#!/bin/bash
# PMC passes (kernel-trace only) over the plain vs BN-on-input ring forward, bs 64 256^2 64->64
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/pmcb
export RDP_NO_BUILD=1
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $line -d $R/gpurun_out/pmcb/set$i -o pmc --output-format csv -- \
    python3 $R/scripts/conv_microbench.py --batch 64 --shapes 0 --variants 0,9 --rounds 1 --reps 3 \
    > $R/gpurun_out/pmcb/set$i.log 2>&1 || { echo "set $i failed"; tail -5 $R/gpurun_out/pmcb/set$i.log; exit 1; }
done < $R/scripts/pmc_sets_bnin.txt
find $R/gpurun_out/pmcb -name "*.csv" | head
python3 $R/scripts/pmc_summary.py $R/gpurun_out/pmcb > $R/gpurun_out/pmcb/summary.txt && cat $R/gpurun_out/pmcb/summary.txt
