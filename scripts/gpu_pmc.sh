#!/bin/bash
# Hardware counters (PMC run: kernel-trace only, no sys/runtime trace), one counter set per line of
# scripts/$PMC_FILE; the profiled program is scripts/conv_microbench.py $MB_ARGS, or $PMC_PROG (a repo-relative
# python script) with $MB_ARGS.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/pmc
export RDP_NO_BUILD=1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/pmc/counters_list.txt 2>&1 || true
for set in "${PMC_SETS[@]:-SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA}"; do :; done
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $line -d $GRAFT_REPO_ROOT/gpurun_out/pmc/set$i -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/${PMC_PROG:-scripts/conv_microbench.py} ${MB_ARGS} > $GRAFT_REPO_ROOT/gpurun_out/pmc/set$i.log 2>&1 || { echo "set $i failed"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/pmc/set$i.log; }
done < $GRAFT_REPO_ROOT/scripts/${PMC_FILE:-pmc_sets.txt}
echo done
