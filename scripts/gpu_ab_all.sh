#!/bin/bash
# kernel tests, then serving A/B, then training A/B (bs 4 and 64), base = ab/_C_base.so vs in-tree
set -o pipefail
cd "$GRAFT_REPO_ROOT"
SKIP_TESTS= TESTS="${TESTS:-tests/test_kernels_gpu.py}" FRAMES=${FRAMES:-400} scripts/gpu_serve_ab.sh || exit $?
SKIP_TESTS=1 BATCHES="${BATCHES:-4 64}" scripts/gpu_ab.sh || exit $?
