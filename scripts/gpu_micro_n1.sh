#!/bin/bash
# Conv variants at the serving batch (N = 1) on the split-K shapes: bm_pref 2 (auto 128x128 8-wave),
# 128 (4-wave), 3 / 256 (256x64 8 / 4-wave), 7 / 8 (split-K ping-pong)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/n1
export RDP_NO_BUILD=1
timeout -k 10 300 python -u scripts/conv_microbench.py --batch 1 --variants 2,128,3,256,7,8 --ws 1 --reps 30 --rounds 5 \
  --shapes 2,3,4,5,6,7,12,13,14,15,16,11 > gpurun_out/n1/micro.jsonl 2>&1 || { tail -5 gpurun_out/n1/micro.jsonl; exit 1; }
cat gpurun_out/n1/micro.jsonl
