#!/bin/bash
# BN+ReLU of the layer under each Up block applied by the upsample (RDP_FUSE_UP_BN): GPU tests and step A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/upbn
export RDP_NO_BUILD=1
timeout -k 10 600 python -u -m pytest tests/test_unet_native_gpu.py tests/test_train_serve_gpu.py -x -q --timeout 240 \
  --timeout-method thread > gpurun_out/upbn/tests.log 2>&1
rc=$?; tail -3 gpurun_out/upbn/tests.log; [ $rc -eq 0 ] || exit $rc
run() {  # batch steps tag env...
  local b=$1 st=$2 tag=$3; shift 3
  env "$@" timeout -k 10 300 python bench.py --batch $b --steps $st --warmup 8 --serve 0 --extras 0 \
    > gpurun_out/upbn/b.json 2>> gpurun_out/upbn/bench.err || exit 1
  echo "b$b $tag $(python -c "import json;d=json.load(open('gpurun_out/upbn/b.json'));print(d['value'],d['ms_per_step'])")"
}
for r in 1 2 3; do
  run 4 60 "fuse=0 r$r" RDP_FUSE_UP_BN=0
  run 4 60 "fuse=1 r$r" RDP_FUSE_UP_BN=1
done
for r in 1 2; do
  run 16 30 "fuse=0 r$r" RDP_FUSE_UP_BN=0
  run 16 30 "fuse=1 r$r" RDP_FUSE_UP_BN=1
done
