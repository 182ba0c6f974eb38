#!/bin/bash
# One GPU call: GPU tests, default bench (with extras + serving), eager baseline (archived).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export RDP_NO_BUILD=1
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 ${T:-900} python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -12 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 400 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
  cat gpurun_out/bench.json
fi
if [ -n "$EAGER" ]; then
  for b in 32 4; do
    timeout -k 10 400 python bench.py --impl eager --batch $b --steps 20 --warmup 5 --serve 0 --extras 0 > gpurun_out/eager_b$b.json 2> gpurun_out/eager_b$b.err || { tail -20 gpurun_out/eager_b$b.err; exit 1; }
    cat gpurun_out/eager_b$b.json
  done
fi
