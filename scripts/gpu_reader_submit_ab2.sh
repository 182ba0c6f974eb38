#!/bin/bash
# Reader-thread submit, second A/B: one stream only (streamed FPS + 2,000 lock-step round trips), 5 interleaved
# rounds, to settle the lock-step tail (hybrid: the reader submits only while earlier frames are unanswered).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export RDP_NO_BUILD=1
RDP_SERVE_READER_SUBMIT=1 timeout -k 10 400 python -u -m pytest tests/test_serve_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/rs_tests2.log 2>&1 || { tail -30 gpurun_out/rs_tests2.log; exit 1; }
cat > /tmp/rsab2.py <<'PY'
import json, sys, torch
sys.path.insert(0, ".")
from robotic_discovery_platform_amd.serve.bench_serve import prepare_model, measure_e2e
m, sc = prepare_model(torch.device("cuda"), 50)
r1 = measure_e2e(m, sc, 2000, 50, streams=1)
r1.update(measure_e2e(m, sc, 1000, 50, streams=4))
print(json.dumps({k: v for k, v in r1.items() if k in ("e2e_fps", "e2e_p50_ms", "e2e_p99_ms", "e2e_p999_ms", "e2e_slow_frames", "e2e_fps_4streams")}), flush=True)
import os; os._exit(0)
PY
: > gpurun_out/rs_ab2.txt
for r in 1 2 3 4 5; do for v in 0 1; do
  RDP_SERVE_READER_SUBMIT=$v timeout -k 10 300 python /tmp/rsab2.py > gpurun_out/rs_one.json 2>> gpurun_out/rs_ab2.err || exit 1
  echo "r$r reader_submit=$v $(cat gpurun_out/rs_one.json)" | tee -a gpurun_out/rs_ab2.txt
done; done
