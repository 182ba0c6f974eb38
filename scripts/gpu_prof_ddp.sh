#!/bin/bash
# Kernel trace of the forced-DDP (1-rank RCCL) training step: all-reduce vs wgrad overlap.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export RDP_NO_BUILD=1
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for c in ${COMMS:-fp32 bf16}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_ddp_$c -o ddp --output-format csv -- python3 $R/bench.py --batch ${B:-64} --steps 4 --warmup 2 --serve 0 --ddp-force 1 --grad-comm $c > $R/gpurun_out/prof_ddp_$c.log 2>&1 || { tail -30 $R/gpurun_out/prof_ddp_$c.log; exit 1; }
  tail -1 $R/gpurun_out/prof_ddp_$c.log
  f=$(find $R/gpurun_out/prof_ddp_$c -name '*kernel_trace.csv' | head -1)
  python3 $R/scripts/comm_overlap.py $f 3 > $R/gpurun_out/overlap_$c.txt 2>&1; cat $R/gpurun_out/overlap_$c.txt | tail -30
done
