#!/bin/bash
# Full GPU validation (GPU tests, default bench) followed by the bs-64 / bs-4 step and serving kernel traces.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && bash scripts/gpu_ab.sh && bash scripts/gpu_final_profiles.sh
