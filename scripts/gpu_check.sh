#!/bin/bash
# One GPU call: the GPU test suite, smoke(), then the default bench and the reference-batch bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export RDP_NO_BUILD=1
timeout -k 10 ${T:-900} python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
if [ -n "$BENCH" ]; then
  timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
  cat gpurun_out/bench_default.json
  timeout -k 10 300 python bench.py --batch 4 --steps 50 --warmup 10 --serve 0 > gpurun_out/bench_b4.json 2> gpurun_out/bench_b4.err || { tail -20 gpurun_out/bench_b4.err; exit 1; }
  cat gpurun_out/bench_b4.json
fi
