#!/bin/bash
# One GPU call: the GPU test suite, then the default bench and the reference-batch bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export RDP_NO_BUILD=1
timeout -k 10 ${T:-900} python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
if [ -n "$BENCH" ]; then
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_b64.json 2> gpurun_out/bench_b64.err || { tail -20 gpurun_out/bench_b64.err; exit 1; }
  cat gpurun_out/bench_b64.json
  timeout -k 10 300 python bench.py --batch 4 --steps 50 --warmup 10 --serve 0 > gpurun_out/bench_b4.json 2> gpurun_out/bench_b4.err || { tail -20 gpurun_out/bench_b4.err; exit 1; }
  cat gpurun_out/bench_b4.json
fi
