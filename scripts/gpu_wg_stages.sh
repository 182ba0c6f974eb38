#!/bin/bash
# halo wgrad pipeline depth A/B in isolation (RDP_WGRAD_HALO_STAGES is read once per process)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export RDP_NO_BUILD=1
for st in 2 3; do
  RDP_WGRAD_HALO_STAGES=$st timeout -k 10 300 python -u scripts/conv_microbench.py --wgrad --batch 64 --shapes 2,3,7 --variants 0,5 --rounds 5 --wgrad-blocks 512 > gpurun_out/wg_st$st.log 2>&1 || { tail -20 gpurun_out/wg_st$st.log; exit 1; }
  echo "stages=$st"; tail -3 gpurun_out/wg_st$st.log
done
