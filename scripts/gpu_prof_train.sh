#!/bin/bash
# rocprofv3 kernel traces: bs-64 training step (default schedule + serialised), serving frames.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export RDP_NO_BUILD=1
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_train -o train --output-format csv -- python3 $R/bench.py --batch 64 --steps 4 --warmup 3 --serve 0 --extras 0 > $R/gpurun_out/prof_train.log 2>&1 || { tail -20 $R/gpurun_out/prof_train.log; exit 1; }
echo train_ok
RDP_WGRAD_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_serial -o serial --output-format csv -- python3 $R/bench.py --batch 64 --steps 4 --warmup 3 --serve 0 --extras 0 > $R/gpurun_out/prof_serial.log 2>&1 || { tail -20 $R/gpurun_out/prof_serial.log; exit 1; }
echo serial_ok
