#!/bin/bash
# Batched serving check: kernel + batch tests, per-batch GPU time, engine pipelined 2 / 4 / 8 streams (2 rounds).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export RDP_NO_BUILD=1
timeout -k 10 400 python -u -m pytest tests/test_serve_batch_gpu.py "tests/test_kernels_gpu.py::test_conv_eval_fused_pool" "tests/test_kernels_gpu.py::test_conv_eval_fused_upsample" tests/test_serve_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/batch_tests.log 2>&1 || { tail -30 gpurun_out/batch_tests.log; exit 1; }
tail -2 gpurun_out/batch_tests.log
timeout -k 10 200 python scripts/serve_batch_bench.py --reps 100 > gpurun_out/sb.json 2>> gpurun_out/sb.err || exit 1
cat gpurun_out/sb.json
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
for r in 1 2; do for v in "X=1" "RDP_BATCH_PRE=0"; do
  env $v timeout -k 10 300 python /tmp/pipe.py > gpurun_out/pipe.json 2>> gpurun_out/sb.err || exit 1
  echo "r$r $v $(cat gpurun_out/pipe.json)" | tee -a gpurun_out/batch_check.txt
done; done
