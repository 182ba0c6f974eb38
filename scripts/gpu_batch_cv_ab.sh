#!/bin/bash
# BatchEngine wake-ups: one condition per event (default) vs one shared condition (RDP_BATCH_ONECV=1), interleaved:
# engine pipelined 4 / 8 streams and e2e gRPC 4 streams. Batch tests first.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export RDP_NO_BUILD=1
timeout -k 10 400 python -u -m pytest tests/test_serve_batch_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/cv_tests.log 2>&1 || { tail -30 gpurun_out/cv_tests.log; exit 1; }
tail -2 gpurun_out/cv_tests.log
cat > /tmp/cvab.py <<'PY'
import json, sys, torch
sys.path.insert(0, ".")
from robotic_discovery_platform_amd.serve.bench_serve import prepare_model, measure_engine_pipelined, measure_e2e
m, sc = prepare_model(torch.device("cuda"), 50)
out = {}
for st in (4, 8):
    out.update(measure_engine_pipelined(m, sc, 1000, 50, streams=st))
r = measure_e2e(m, sc, 1000, 50, streams=4)
out.update({k: v for k, v in r.items() if k in ("e2e_fps_4streams", "e2e_stage_gpu_p50_ms_4streams")})
print(json.dumps({k: v for k, v in out.items() if "batch_sizes" not in k}), flush=True)
import os; os._exit(0)
PY
: > gpurun_out/cv_ab.txt
for r in 1 2 3; do for v in 0 1; do
  RDP_BATCH_ONECV=$v timeout -k 10 300 python /tmp/cvab.py > gpurun_out/cv_one.json 2>> gpurun_out/cv_ab.err || exit 1
  echo "r$r onecv=$v $(cat gpurun_out/cv_one.json)" | tee -a gpurun_out/cv_ab.txt
done; done
