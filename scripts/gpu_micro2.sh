#!/bin/bash
# Labelled conv microbench (fwd auto, wgrad at the isolated and the in-step split targets) + serving bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export RDP_NO_BUILD=1
timeout -k 10 300 python scripts/conv_microbench.py --variants 0 --rounds 3 --out gpurun_out/mb_fwd.json > gpurun_out/mb_fwd.log 2>&1 || { tail gpurun_out/mb_fwd.log; exit 1; }
timeout -k 10 300 python scripts/conv_microbench.py --wgrad --variants 0 --rounds 3 --wgrad-blocks 2048 --out gpurun_out/mb_wg2048.json > gpurun_out/mb_wg2048.log 2>&1 || { tail gpurun_out/mb_wg2048.log; exit 1; }
timeout -k 10 300 python scripts/conv_microbench.py --wgrad --variants 0 --rounds 3 --wgrad-blocks 512 --out gpurun_out/mb_wg512.json > gpurun_out/mb_wg512.log 2>&1 || { tail gpurun_out/mb_wg512.log; exit 1; }
echo micro_ok
if [ -n "$SERVE" ]; then
  timeout -k 10 400 python -m robotic_discovery_platform_amd.serve.bench_serve --frames 300 --warmup 30 --train-steps 200 > gpurun_out/serve_full2.json 2> gpurun_out/serve_full2.err || { tail -20 gpurun_out/serve_full2.err; exit 1; }
  cat gpurun_out/serve_full2.json
fi
