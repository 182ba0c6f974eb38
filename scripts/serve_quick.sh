set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export RDP_NO_BUILD=1 PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_serve_gpu.py tests/test_serve_replicas_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_serve.log 2>&1 || { tail -30 gpurun_out/pytest_serve.log; exit 1; }
tail -1 gpurun_out/pytest_serve.log
timeout -k 10 200 python scripts/serve_host_timing.py > gpurun_out/host_timing.jsonl 2>/dev/null || exit 1
cat gpurun_out/host_timing.jsonl
timeout -k 10 300 python -m robotic_discovery_platform_amd.serve.bench_serve --frames 300 --warmup 30 --e2e 1 > gpurun_out/serve_full.json 2> gpurun_out/serve_full.err || { tail -5 gpurun_out/serve_full.err; exit 1; }
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ev3/prof_serve -o serve --output-format csv -- python3 -m robotic_discovery_platform_amd.serve.bench_serve --frames 200 --warmup 20 --train-steps 200 --e2e 0 --multi 0 > $R/gpurun_out/ev3_prof_serve.log 2>&1 || { tail -5 $R/gpurun_out/ev3_prof_serve.log; exit 1; }
echo done
