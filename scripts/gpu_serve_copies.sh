#!/bin/bash
# Serving engine frames with kernel + memory-copy traces (where the GPU time outside the kernels goes).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R"; mkdir -p gpurun_out/scopy
export RDP_NO_BUILD=1 PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $R/gpurun_out/scopy/prof -o serve --output-format csv -- python3 -m robotic_discovery_platform_amd.serve.bench_serve --frames 120 --warmup 20 --train-steps 20 --e2e 0 --multi 0 > $R/gpurun_out/scopy/prof.log 2>&1 || { tail -20 $R/gpurun_out/scopy/prof.log; exit 1; }
ls $R/gpurun_out/scopy/prof
