#!/bin/bash
# Batched serving round 2: batched-geometry correctness + per-batch GPU time (geo batched vs per-frame) + pipelined A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export RDP_NO_BUILD=1
timeout -k 10 300 python -u -m pytest tests/test_serve_batch_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/batch_tests.log 2>&1 || { tail -30 gpurun_out/batch_tests.log; exit 1; }
tail -2 gpurun_out/batch_tests.log
: > gpurun_out/batch_ab2.txt
for v in "RDP_BATCH_UPLOAD=kernel" "RDP_BATCH_UPLOAD=kernel RDP_BATCH_GEO=0" "X=1"; do
  env $v timeout -k 10 200 python scripts/serve_batch_bench.py --reps 100 > gpurun_out/sb.json 2>> gpurun_out/sb.err || exit 1
  echo "$v $(cat gpurun_out/sb.json)" | tee -a gpurun_out/batch_ab2.txt
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_batch2 -o run -- python3 scripts/serve_batch_bench.py --reps 30 --sizes 4 > gpurun_out/serve_batch_prof.json 2>> gpurun_out/sb.err || exit 1
cat > /tmp/pipe.py <<'PY'
import json, sys, torch
sys.path.insert(0, ".")
from robotic_discovery_platform_amd.serve.bench_serve import prepare_model, measure_engine_pipelined
m, sc = prepare_model(torch.device("cuda"), 50)
out = {}
for st in (2, 4, 8):
    out.update(measure_engine_pipelined(m, sc, 1000, 50, streams=st))
print(json.dumps(out), flush=True)
import os; os._exit(0)
PY
for r in 1 2; do for v in "RDP_BATCH_UPLOAD=kernel" "X=1" "RDP_SERVE_BATCH=0"; do
  env $v timeout -k 10 300 python /tmp/pipe.py > gpurun_out/pipe.json 2>> gpurun_out/sb.err || exit 1
  echo "r$r $v $(cat gpurun_out/pipe.json)" | tee -a gpurun_out/batch_ab2.txt
done; done
