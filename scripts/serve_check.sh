#!/bin/bash
# Serving GPU check: the serving GPU tests (NOTESTS=1 skips them), then either an interleaved A/B of
# AB="ENV=v1 ENV=v2" settings (engine + E2E=1 gRPC rows, 2 rounds) or the e2e topology sweep.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export RDP_NO_BUILD=1
if [ -z "$NOTESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_serve_gpu.py tests/test_serve_replicas_gpu.py tests/test_train_serve_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_serve.log 2>&1 || { tail -30 gpurun_out/pytest_serve.log; exit 1; }
  tail -3 gpurun_out/pytest_serve.log
fi
if [ -n "$AB" ]; then
  for r in 1 2; do for e in $AB; do
    env ${e//,/ } timeout -k 10 400 python -m robotic_discovery_platform_amd.serve.bench_serve --frames 400 --warmup 40 --e2e ${E2E:-0} --multi 1 > gpurun_out/sab.json 2> gpurun_out/sab.err || { tail -20 gpurun_out/sab.err; exit 1; }
    python -c "
import json;d=json.loads(open('gpurun_out/sab.json').read().splitlines()[-1])
print('$e r$r', {k: d[k] for k in sorted(d) if k.startswith('serve_') and isinstance(d[k], (int, float)) and not k.endswith('p99_ms')})"
  done; done
else
  timeout -k 10 400 python scripts/serve_e2e_ab.py --switch 0 --streams ${STREAMS:-1,4,8} --procs ${PROCS:-2:4,4:4,4:8,8:8} > gpurun_out/e2e_ab2.jsonl 2> gpurun_out/e2e_ab2.err
fi
