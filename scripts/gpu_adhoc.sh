set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export RDP_NO_BUILD=1
timeout -k 10 300 python scripts/conv_microbench.py --variants 3,10003,0,10000 --rounds 5 --shapes 1,2,3,4,6,7,8,9 > gpurun_out/micro_f.log 2>&1 || { tail -20 gpurun_out/micro_f.log; exit 1; }
cat gpurun_out/micro_f.log
