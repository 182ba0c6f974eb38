#!/bin/bash
# Raw request bytes (native payload parse) vs protobuf-parsed requests: serving GPU tests, then e2e 1 / 4 streams.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export RDP_NO_BUILD=1
timeout -k 10 500 python -u -m pytest tests/test_serve_gpu.py tests/test_serve_replicas_gpu.py tests/test_serve_batch_gpu.py tests/test_train_serve_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/raw_tests.log 2>&1 || { tail -30 gpurun_out/raw_tests.log; exit 1; }
tail -2 gpurun_out/raw_tests.log
cat > /tmp/e2e.py <<'PY'
import json, sys, torch
sys.path.insert(0, ".")
from robotic_discovery_platform_amd.serve.bench_serve import prepare_model, measure_e2e
m, sc = prepare_model(torch.device("cuda"), 50)
out = {}
out.update({k: v for k, v in measure_e2e(m, sc, 1000, 50).items() if k in ("e2e_fps", "e2e_p50_ms", "e2e_p99_ms")})
out.update({k: v for k, v in measure_e2e(m, sc, 1000, 50, streams=4).items() if "fps" in k or "gpu_p50" in k})
print(json.dumps(out), flush=True)
import os; os._exit(0)
PY
: > gpurun_out/raw_ab.txt
for r in 1 2; do for v in "RDP_SERVE_RAW=1" "RDP_SERVE_RAW=0"; do
  env $v timeout -k 10 300 python /tmp/e2e.py > gpurun_out/e2e.json 2>> gpurun_out/e2e.err || exit 1
  echo "r$r $v $(cat gpurun_out/e2e.json)" | tee -a gpurun_out/raw_ab.txt
done; done
