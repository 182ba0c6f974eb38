#!/bin/bash
# MFMA busy and kernel time per served frame: the batched serving network at n = 1 vs n = 4 frames per batch
# (BatchEngine graph replays, scripts/serve_batch_bench.py --single 0), one rocprofv3 --pmc pass each
# (kernel trace only). Summarised by scripts/pmc_batch.py.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R"; mkdir -p gpurun_out/pmcb
export RDP_NO_BUILD=1 PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
for n in 1 4; do
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES \
    -d $R/gpurun_out/pmcb/n$n -o pmc --output-format csv -- python3 $R/scripts/serve_batch_bench.py --sizes $n --single 0 --reps 100 \
    > $R/gpurun_out/pmcb/n$n.log 2>&1 || { echo "n=$n failed"; tail -20 $R/gpurun_out/pmcb/n$n.log; exit 1; }
done
cd "$R" && python3 scripts/pmc_batch.py gpurun_out/pmcb | tee gpurun_out/pmcb/summary.md
