#!/bin/bash
# train_model throughput (bench extras) A/B of the fused first-layer wgrad, 3 interleaved rounds
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export RDP_NO_BUILD=1
for round in 1 2 3; do
for v in 0 1; do
  RDP_FUSE_FIRST_WGRAD=$v timeout -k 10 300 python bench.py --steps 5 --warmup 2 --serve 0 --extras 1 > gpurun_out/tm_${v}_$round.json 2> gpurun_out/tm_${v}_$round.err || { tail -20 gpurun_out/tm_${v}_$round.err; exit 1; }
  echo "fuse=$v round$round $(python3 -c "import json;d=json.load(open('gpurun_out/tm_${v}_$round.json'));print(d['value'], d['ref_batch_imgs_per_s'], d['train_model_imgs_per_s'], d['train_model_epoch_s'])")"
done
done
