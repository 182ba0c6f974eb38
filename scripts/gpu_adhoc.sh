set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export RDP_NO_BUILD=1
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_serve_gpu.py tests/test_serve_cpu.py > gpurun_out/t_s.log 2>&1 || { tail -30 gpurun_out/t_s.log; exit 1; }
tail -1 gpurun_out/t_s.log
for i in 1 2; do
timeout -k 10 300 python -m robotic_discovery_platform_amd.serve.bench_serve > gpurun_out/serve.json 2> gpurun_out/serve.err || { tail -20 gpurun_out/serve.err; exit 1; }
tail -1 gpurun_out/serve.json
done
