#!/bin/bash
# Serving: GPU tests, engine variants (split-K on/off), full serving bench, one-frame kernel timeline.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export RDP_NO_BUILD=1
R=$GRAFT_REPO_ROOT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_serve_gpu.py tests/test_geo_spline_gpu.py tests/test_train_serve_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_serve.log 2>&1
  rc=$?; tail -4 gpurun_out/pytest_serve.log; [ $rc -eq 0 ] || exit $rc
fi
for sk in 1 0; do
  RDP_SPLITK=$sk timeout -k 10 300 python -m robotic_discovery_platform_amd.serve.bench_serve --frames 300 --warmup 30 --train-steps 20 --e2e 0 > gpurun_out/serve_splitk$sk.json 2> gpurun_out/serve_splitk$sk.err || { tail -20 gpurun_out/serve_splitk$sk.err; exit 1; }
  echo "splitk=$sk $(cat gpurun_out/serve_splitk$sk.json)"
done
timeout -k 10 300 python -m robotic_discovery_platform_amd.serve.bench_serve --frames 300 --warmup 30 --train-steps 200 > gpurun_out/serve_full.json 2> gpurun_out/serve_full.err || { tail -20 gpurun_out/serve_full.err; exit 1; }
cat gpurun_out/serve_full.json
export PYTHONPATH=$R; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_serve -o serve --output-format csv -- python3 -m robotic_discovery_platform_amd.serve.bench_serve --frames 60 --warmup 10 --train-steps 5 --e2e 0 > $R/gpurun_out/prof_serve.log 2>&1 || { tail -20 $R/gpurun_out/prof_serve.log; exit 1; }
f=$(find $R/gpurun_out/prof_serve -name '*kernel_trace.csv' | head -1)
python3 $R/scripts/serve_frame.py $f > $R/gpurun_out/serve_frame.txt; tail -45 $R/gpurun_out/serve_frame.txt
