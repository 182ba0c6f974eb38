#!/bin/bash
# Reader-thread submit of encoded frames (serve/server.py _analyze_pipelined) vs the handler submit
# (RDP_SERVE_READER_SUBMIT=0): serving GPU tests, then e2e gRPC 1 stream (streamed FPS + lock-step latency)
# and 4 streams, interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export RDP_NO_BUILD=1
RDP_SERVE_READER_SUBMIT=1 timeout -k 10 500 python -u -m pytest tests/test_serve_gpu.py tests/test_serve_batch_gpu.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/rs_tests.log 2>&1 || { tail -30 gpurun_out/rs_tests.log; exit 1; }
tail -2 gpurun_out/rs_tests.log
cat > /tmp/rsab.py <<'PY'
import json, sys, torch
sys.path.insert(0, ".")
from robotic_discovery_platform_amd.serve.bench_serve import prepare_model, measure_e2e
m, sc = prepare_model(torch.device("cuda"), 50)
out = {}
r1 = measure_e2e(m, sc, 2000, 50, streams=1)
out.update({k: v for k, v in r1.items() if k in ("e2e_fps", "e2e_p50_ms", "e2e_p99_ms", "e2e_stage_submit_p50_ms")})
r4 = measure_e2e(m, sc, 1000, 50, streams=4)
out.update({k: v for k, v in r4.items() if k in ("e2e_fps_4streams",)})
print(json.dumps(out), flush=True)
import os; os._exit(0)
PY
: > gpurun_out/rs_ab.txt
for r in 1 2 3; do for v in 0 1; do
  RDP_SERVE_READER_SUBMIT=$v timeout -k 10 300 python /tmp/rsab.py > gpurun_out/rs_one.json 2>> gpurun_out/rs_ab.err || exit 1
  echo "r$r reader_submit=$v $(cat gpurun_out/rs_one.json)" | tee -a gpurun_out/rs_ab.txt
done; done
