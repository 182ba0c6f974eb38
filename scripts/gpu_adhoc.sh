set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export RDP_NO_BUILD=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_unet_native_gpu.py > gpurun_out/t_unet.log 2>&1 || { tail -30 gpurun_out/t_unet.log; exit 1; }
tail -2 gpurun_out/t_unet.log
timeout -k 10 300 python bench.py --batch 32 --steps 20 --warmup 5 --serve 0 > gpurun_out/b32.json 2> gpurun_out/b32.err || { tail -20 gpurun_out/b32.err; exit 1; }
cat gpurun_out/b32.json
timeout -k 10 300 python bench.py --batch 64 --steps 10 --warmup 3 --serve 0 > gpurun_out/b64.json 2> gpurun_out/b64.err || { tail -20 gpurun_out/b64.err; exit 1; }
cat gpurun_out/b64.json
