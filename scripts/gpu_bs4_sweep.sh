#!/bin/bash
# Reference-batch (bs 4) conv variant sweep: every U-Net fwd / dgrad shape under each dispatch variant
# (bm_pref: 0 auto, 2 igemm 128x128 8-wave, 3 igemm 256x64 8-wave, 4 / 5 ping-pong 256x256 / 256x128,
# 7 / 8 split-K ping-pong, 128 / 256 igemm 4-wave; +1000k: k blocks per CU), with the split-K workspace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export RDP_NO_BUILD=1
timeout -k 10 300 python scripts/conv_microbench.py --batch 4 --ws 1 --rounds 7 --reps 20 \
  --variants 0,2,3,4,5,7,8,128,256,1002,4002,8002 --out gpurun_out/bs4_sweep.json > gpurun_out/bs4_sweep.log 2>&1
rc=$?
tail -30 gpurun_out/bs4_sweep.log
exit $rc
