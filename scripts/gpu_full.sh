#!/bin/bash
# Full GPU test suite + default bench (extras + serving) + transposed-decoder bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export RDP_NO_BUILD=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 300 python bench.py --decoder transposed --serve 0 --extras 0 > gpurun_out/bench_tr.json 2> gpurun_out/bench_tr.err || { tail -20 gpurun_out/bench_tr.err; exit 1; }
cat gpurun_out/bench_tr.json
timeout -k 10 300 python bench.py --batch 256 --steps 5 --warmup 2 --serve 0 --extras 0 > gpurun_out/bench_b256.json 2> gpurun_out/bench_b256.err || { tail -20 gpurun_out/bench_b256.err; exit 1; }
cat gpurun_out/bench_b256.json
