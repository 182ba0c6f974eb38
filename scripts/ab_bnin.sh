set -o pipefail
cd "$GRAFT_REPO_ROOT"; export RDP_NO_BUILD=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "bnin" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_bnin.log 2>&1 || { tail -30 gpurun_out/pytest_bnin.log; exit 1; }
tail -1 gpurun_out/pytest_bnin.log
timeout -k 10 400 python -u -m pytest tests/test_unet_native_gpu.py tests/test_ddp_rccl_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_unet.log 2>&1 || { tail -30 gpurun_out/pytest_unet.log; exit 1; }
tail -1 gpurun_out/pytest_unet.log
for r in 1 2; do for ab in 0 1; do for b in 64 4; do
RDP_AB_BNIN=$ab timeout -k 10 200 python bench.py --batch $b --steps 30 --warmup 5 --serve 0 --extras 0 > gpurun_out/bnin_${ab}_b${b}_$r.json 2> gpurun_out/bnin.err || exit 1
done; done; done
