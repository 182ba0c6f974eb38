set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export RDP_NO_BUILD=1
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_serve_gpu.py > gpurun_out/t_s.log 2>&1 || { tail -30 gpurun_out/t_s.log; exit 1; }
tail -1 gpurun_out/t_s.log
cd /tmp && export TMPDIR=/tmp
PYTHONPATH=$R timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_serve -o serve --output-format csv -- python3 -m robotic_discovery_platform_amd.serve.bench_serve --frames 200 --warmup 20 --train-steps 20 > $R/gpurun_out/prof_serve.log 2>&1 || { tail -20 $R/gpurun_out/prof_serve.log; exit 1; }
cd $R
timeout -k 10 300 python -m robotic_discovery_platform_amd.serve.bench_serve > gpurun_out/serve.json 2> gpurun_out/serve.err || { tail -20 gpurun_out/serve.err; exit 1; }
tail -3 gpurun_out/serve.json
