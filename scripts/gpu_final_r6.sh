#!/bin/bash
# Round 6 closing run: the full GPU suite on this commit, then the driver's default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export RDP_NO_BUILD=1
git_head=$(cat .git_head 2>/dev/null || echo unknown)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_final.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_gpu_final.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { tail -20 gpurun_out/bench_final.err; exit 1; }
tail -1 gpurun_out/bench_final.json | cut -c1-400
