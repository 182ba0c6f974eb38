#!/bin/bash
# Round 6: full GPU suite + the world-1 DDP bench self-check (native probe, forced fallback).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export RDP_NO_BUILD=1
timeout -k 10 ${T:-900} python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS} \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --ddp-force 1 --steps 5 --warmup 3 --extras 0 --serve 0 > gpurun_out/bench_ddp1.json 2> gpurun_out/bench_ddp1.err || exit $?
cat gpurun_out/bench_ddp1.json
RDP_COMM_PROBE_FAIL=1 timeout -k 10 300 python bench.py --ddp-force 1 --steps 5 --warmup 3 --extras 0 --serve 0 > gpurun_out/bench_ddp1_fail.json 2> gpurun_out/bench_ddp1_fail.err || exit $?
cat gpurun_out/bench_ddp1_fail.json
