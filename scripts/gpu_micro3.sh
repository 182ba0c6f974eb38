#!/bin/bash
# Labelled conv microbench at bs 64: auto dispatch with / without the ping-pong kernel, wgrad (512 blocks).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export RDP_NO_BUILD=1
timeout -k 10 300 python scripts/conv_microbench.py --batch 64 --variants 0 --rounds 3 --out gpurun_out/mb_fwd_pp.json > gpurun_out/mb_fwd_pp.log 2>&1 || { tail gpurun_out/mb_fwd_pp.log; exit 1; }
RDP_CONV_PP=0 timeout -k 10 300 python scripts/conv_microbench.py --batch 64 --variants 0 --rounds 3 --out gpurun_out/mb_fwd_nopp.json > gpurun_out/mb_fwd_nopp.log 2>&1 || { tail gpurun_out/mb_fwd_nopp.log; exit 1; }
timeout -k 10 300 python scripts/conv_microbench.py --batch 64 --wgrad --variants 0 --rounds 3 --wgrad-blocks 512 --out gpurun_out/mb_wg512.json > gpurun_out/mb_wg512.log 2>&1 || { tail gpurun_out/mb_wg512.log; exit 1; }
echo micro_ok
