#!/bin/bash
# GPU numerics tests (one pytest process), each step under its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export RDP_NO_BUILD=1
timeout -k 10 ${T:-600} python -m pytest tests -m gpu -x -q ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -40 gpurun_out/pytest_gpu.log
exit $rc
