set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export RDP_NO_BUILD=1
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "head" > gpurun_out/t_f.log 2>&1 || { tail -30 gpurun_out/t_f.log; exit 1; }
tail -1 gpurun_out/t_f.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_unet_native_gpu.py > gpurun_out/t_u.log 2>&1 || { tail -30 gpurun_out/t_u.log; exit 1; }
tail -1 gpurun_out/t_u.log
RDP_FUSE_HEAD=0 timeout -k 10 400 python bench.py --serve 0 > gpurun_out/b64_nofuse.json 2> gpurun_out/b64_nofuse.err || { tail -20 gpurun_out/b64_nofuse.err; exit 1; }
cat gpurun_out/b64_nofuse.json
timeout -k 10 400 python bench.py --serve 0 > gpurun_out/b64.json 2> gpurun_out/b64.err || { tail -20 gpurun_out/b64.err; exit 1; }
cat gpurun_out/b64.json
