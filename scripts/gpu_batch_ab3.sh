#!/bin/bash
# Batched serving round 3: lanes (concurrent batch streams) 1 vs 2 vs unbatched; engine pipelined + e2e 4 streams.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export RDP_NO_BUILD=1
timeout -k 10 300 python -u -m pytest tests/test_serve_batch_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/batch_tests.log 2>&1 || { tail -30 gpurun_out/batch_tests.log; exit 1; }
tail -2 gpurun_out/batch_tests.log
: > gpurun_out/batch_ab3.txt
cat > /tmp/pipe.py <<'PY'
import json, sys, torch
sys.path.insert(0, ".")
from robotic_discovery_platform_amd.serve.bench_serve import prepare_model, measure_engine_pipelined, measure_e2e
m, sc = prepare_model(torch.device("cuda"), 50)
out = {}
for st in (1, 2, 4, 8):
    out.update(measure_engine_pipelined(m, sc, 1000, 50, streams=st))
out.update({k: v for k, v in measure_e2e(m, sc, 1000, 50, streams=4).items() if "fps" in k or "gpu_p50" in k})
print(json.dumps(out), flush=True)
import os; os._exit(0)
PY
for r in 1 2; do for v in "RDP_BATCH_LANES=1" "RDP_BATCH_LANES=2" "RDP_SERVE_BATCH=0"; do
  env $v timeout -k 10 300 python /tmp/pipe.py > gpurun_out/pipe.json 2>> gpurun_out/sb.err || exit 1
  echo "r$r $v $(cat gpurun_out/pipe.json)" | tee -a gpurun_out/batch_ab3.txt
done; done
