set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export RDP_NO_BUILD=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_race_screens_gpu.py > gpurun_out/t_k.log 2>&1 || { tail -30 gpurun_out/t_k.log; exit 1; }
tail -2 gpurun_out/t_k.log
timeout -k 10 300 python scripts/conv_microbench.py --variants 0,3,10000 --rounds 3 --shapes 0,1 > gpurun_out/micro_f.log 2>&1 || { tail -20 gpurun_out/micro_f.log; exit 1; }
cat gpurun_out/micro_f.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_unet_native_gpu.py > gpurun_out/t_u.log 2>&1 || { tail -30 gpurun_out/t_u.log; exit 1; }
tail -2 gpurun_out/t_u.log
timeout -k 10 400 python bench.py --serve 0 > gpurun_out/b.json 2> gpurun_out/b.err || { tail -20 gpurun_out/b.err; exit 1; }
cat gpurun_out/b.json
