#!/bin/bash
# wgrad halo kernel ablations (20 = full, 21 = no DMA after prologue, 22 = no MFMA, 24 = no LDS reads, 26 = neither)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export RDP_NO_BUILD=1
timeout -k 10 300 python -u scripts/conv_microbench.py --wgrad --batch 64 --shapes ${SHAPES:-2,3,6} --variants ${VARS:-0,20,21,22,24,26} --rounds 5 --wgrad-blocks 512 > gpurun_out/wg_abl.log 2>&1 || { tail -20 gpurun_out/wg_abl.log; exit 1; }
tail -4 gpurun_out/wg_abl.log
