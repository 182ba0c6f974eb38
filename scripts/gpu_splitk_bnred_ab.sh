#!/bin/bash
# BN-backward partials from the split-K dgrad reduce (RDP_SPLITK_BNRED): kernel + training tests, then the
# reference batch (bs 4) and bs 64 interleaved with the separate bn_relu_bwd_reduce pass.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export RDP_NO_BUILD=1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_unet_native_gpu.py tests/test_race_screens_gpu.py \
  -x -q --timeout 120 --timeout-method thread > gpurun_out/sbn_tests.log 2>&1
rc=$?
tail -3 gpurun_out/sbn_tests.log
[ $rc -ne 0 ] && exit $rc
out=gpurun_out/sbn_ab.txt; : > $out
for r in 1 2 3; do
  for v in 0 1; do
    for bs in 4 64; do
      RDP_SPLITK_BNRED=$v timeout -k 10 240 python bench.py --batch $bs --steps 30 --warmup 8 --serve 0 --extras 0 \
        > gpurun_out/sbn_one.json 2>> gpurun_out/sbn_ab.err || exit 1
      echo "r$r fused=$v bs=$bs $(python -c "import json;d=json.loads(open('gpurun_out/sbn_one.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])")" | tee -a $out
    done
  done
done
