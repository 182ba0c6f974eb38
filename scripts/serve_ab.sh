set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export RDP_NO_BUILD=1 PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_serve_gpu.py tests/test_serve_replicas_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_serve.log 2>&1 || { tail -30 gpurun_out/pytest_serve.log; exit 1; }
tail -1 gpurun_out/pytest_serve.log
for r in 1 2; do for d in 0 1; do
RDP_AB_DSTREAM=$d timeout -k 10 300 python -m robotic_discovery_platform_amd.serve.bench_serve --frames 300 --warmup 30 --e2e 1 > gpurun_out/sab_d${d}_$r.json 2> gpurun_out/sab.err || { tail -5 gpurun_out/sab.err; exit 1; }
done; done
