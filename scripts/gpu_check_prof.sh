#!/bin/bash
# Full GPU validation (tests, smoke, default + bs-4 bench) followed by the bs-64 / bs-4 step kernel traces.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R" && BENCH=1 bash scripts/gpu_check.sh || exit 1
mkdir -p gpurun_out/fin
export RDP_NO_BUILD=1 PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/fin/prof_train -o train --output-format csv -- python3 $R/bench.py --batch 64 --steps 4 --warmup 3 --serve 0 --extras 0 > $R/gpurun_out/fin/prof_train.log 2>&1 || { tail -20 $R/gpurun_out/fin/prof_train.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/fin/prof_bs4 -o bs4 --output-format csv -- python3 $R/bench.py --batch 4 --steps 20 --warmup 5 --serve 0 --extras 0 > $R/gpurun_out/fin/prof_bs4.log 2>&1 || { tail -20 $R/gpurun_out/fin/prof_bs4.log; exit 1; }
echo prof_ok
