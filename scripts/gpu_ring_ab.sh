#!/bin/bash
# A/B of the row-ring grid bound on <= 128-wide maps (csrc/conv_igemm.hip ring_auto_grid): the reference
# batch (bs 4) and the bs-64 step, old bound (256 pairs) vs new (1024), interleaved on one box; then the
# GPU conv / training tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export RDP_NO_BUILD=1
out=gpurun_out/ring_ab.txt; : > $out
for r in 1 2; do
  for b in 256 1024; do
    for bs in 4 64; do
      RDP_RING_W128_PAIRS=$b timeout -k 10 240 python bench.py --batch $bs --steps 30 --warmup 8 --serve 0 --extras 0 \
        > gpurun_out/ring_ab_one.json 2>> gpurun_out/ring_ab.err || exit 1
      echo "r$r pairs=$b bs=$bs $(python -c "import json;d=json.loads(open('gpurun_out/ring_ab_one.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])")" | tee -a $out
    done
  done
done
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_unet_native_gpu.py tests/test_serve_gpu.py \
  -x -q --timeout 120 --timeout-method thread > gpurun_out/ring_tests.log 2>&1
rc=$?
tail -3 gpurun_out/ring_tests.log
exit $rc
