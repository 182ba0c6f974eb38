#!/bin/bash
# train_model (bs 4, on-disk dataset) with / without the heap freeze before the epoch loop, interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export RDP_NO_BUILD=1
cat > /tmp/tm.py <<'PY'
import json, sys, argparse, torch
sys.path.insert(0, ".")
import bench
a = argparse.Namespace(size=256, decoder="bilinear")
print(json.dumps(bench.measure_train_model(a, torch.device("cuda"))), flush=True)
import os; os._exit(0)
PY
: > gpurun_out/tgc_ab.txt
for r in 1 2 3; do for v in 1 0; do
  RDP_TRAIN_GC_FREEZE=$v timeout -k 10 300 python /tmp/tm.py > gpurun_out/tgc_one.json 2>> gpurun_out/tgc_ab.err || exit 1
  echo "r$r freeze=$v $(tail -1 gpurun_out/tgc_one.json)" | tee -a gpurun_out/tgc_ab.txt
done; done
