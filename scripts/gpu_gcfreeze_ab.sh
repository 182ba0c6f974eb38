#!/bin/bash
# bench.py with / without the gc freeze before the timed regions, interleaved on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export RDP_NO_BUILD=1
: > gpurun_out/gc_ab.txt
for r in 1 2; do for v in 1 0; do
  RDP_BENCH_GC_FREEZE=$v timeout -k 10 300 python bench.py --serve 0 > gpurun_out/gc_one.json 2>> gpurun_out/gc_ab.err || exit 1
  echo "r$r freeze=$v $(python -c "import json;d=json.loads(open('gpurun_out/gc_one.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['ref_batch_imgs_per_s'],d['transposed_imgs_per_s'],d['train_model_imgs_per_s'])")" | tee -a gpurun_out/gc_ab.txt
done; done
