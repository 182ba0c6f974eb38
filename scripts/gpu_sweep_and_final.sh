#!/bin/bash
# bs-4 conv variant sweep, then the full GPU suite + the default bench line (scripts/gpu_final_r6.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_bs4_sweep.sh && bash scripts/gpu_final_r6.sh
