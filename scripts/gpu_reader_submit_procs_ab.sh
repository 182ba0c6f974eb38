#!/bin/bash
# Reader-thread submit with 2 server processes x 2 streams (serve_e2e_fps_4streams_2procs), interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export RDP_NO_BUILD=1
cat > /tmp/rsp.py <<'PY'
import json, sys, torch
sys.path.insert(0, ".")
from robotic_discovery_platform_amd.serve.bench_serve import prepare_model, measure_e2e_procs
m, sc = prepare_model(torch.device("cuda"), 50)
print(json.dumps(measure_e2e_procs(m, 1000, 50, procs=2, streams=4)), flush=True)
import os; os._exit(0)
PY
: > gpurun_out/rsp_ab.txt
for r in 1 2 3; do for v in 0 1; do
  RDP_SERVE_READER_SUBMIT=$v timeout -k 10 300 python /tmp/rsp.py > gpurun_out/rsp_one.json 2>> gpurun_out/rsp_ab.err || exit 1
  echo "r$r reader_submit=$v $(tail -1 gpurun_out/rsp_one.json | cut -c1-200)" | tee -a gpurun_out/rsp_ab.txt
done; done
