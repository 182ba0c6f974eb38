#!/bin/bash
# rocprofv3 kernel traces: bs-64 training step (default schedule + serialised), serving frames.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export RDP_NO_BUILD=1
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_serve -o serve --output-format csv -- python3 -m robotic_discovery_platform_amd.serve.bench_serve --frames 200 --warmup 20 --train-steps 200 --e2e 0 > $R/gpurun_out/prof_serve.log 2>&1 || { tail -20 $R/gpurun_out/prof_serve.log; exit 1; }
echo serve_ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_bs4 -o bs4 --output-format csv -- python3 $R/bench.py --batch 4 --steps 20 --warmup 5 --serve 0 --extras 0 > $R/gpurun_out/prof_bs4.log 2>&1 || { tail -20 $R/gpurun_out/prof_bs4.log; exit 1; }
echo bs4_ok
