set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export RDP_NO_BUILD=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_race_screens_gpu.py -k "wgrad" > gpurun_out/t_wgrad.log 2>&1 || { tail -30 gpurun_out/t_wgrad.log; exit 1; }
tail -3 gpurun_out/t_wgrad.log
timeout -k 10 300 python scripts/conv_microbench.py --wgrad --variants 4,5 --rounds 3 --shapes 0,1,2,3,7,8,9 > gpurun_out/micro_wg.log 2>&1 || { tail -20 gpurun_out/micro_wg.log; exit 1; }
cat gpurun_out/micro_wg.log
