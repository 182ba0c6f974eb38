#!/bin/bash
# Standalone cost of the BN-on-input row-ring kernels vs the plain ring kernels (64 -> 64, 256^2, bs 64)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/bnin
export RDP_NO_BUILD=1
timeout -k 10 200 python -u scripts/conv_microbench.py --batch 64 --shapes 0 --variants 0,9 --rounds 5 --reps 10 > gpurun_out/bnin/fwd.jsonl 2>&1 || { tail gpurun_out/bnin/fwd.jsonl; exit 1; }
timeout -k 10 200 python -u scripts/conv_microbench.py --batch 64 --shapes 0,9 --variants 0,9 --wgrad --wgrad-blocks 512 --rounds 5 --reps 10 > gpurun_out/bnin/wgrad.jsonl 2>&1 || { tail gpurun_out/bnin/wgrad.jsonl; exit 1; }
grep -v amdgpu.ids gpurun_out/bnin/fwd.jsonl gpurun_out/bnin/wgrad.jsonl
