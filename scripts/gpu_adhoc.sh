set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export RDP_NO_BUILD=1
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_race_screens_gpu.py tests/test_unet_native_gpu.py > gpurun_out/t_k.log 2>&1 || { tail -30 gpurun_out/t_k.log; exit 1; }
tail -1 gpurun_out/t_k.log
timeout -k 10 400 python bench.py --serve 0 > gpurun_out/b64.json 2> gpurun_out/b64.err || { tail -20 gpurun_out/b64.err; exit 1; }
cat gpurun_out/b64.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_graph -o graph --output-format csv -- python3 $R/bench.py --batch 64 --steps 4 --warmup 3 --serve 0 > $R/gpurun_out/prof_graph.log 2>&1 || { tail -20 $R/gpurun_out/prof_graph.log; exit 1; }
cd $R
python scripts/graph_gaps.py gpurun_out/prof_graph/graph_kernel_trace.csv || true
