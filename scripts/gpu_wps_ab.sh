#!/bin/bash
# dgrad weight re-layout on the wgrad side stream after Adam (RDP_WPREP_SIDE): GPU tests, step A/B at bs 4 / 64
set -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R"; mkdir -p gpurun_out/wps
export RDP_NO_BUILD=1
timeout -k 10 600 python -u -m pytest tests/test_unet_native_gpu.py tests/test_train_serve_gpu.py tests/test_ddp_native_gpu.py \
  tests/test_syncbn_native_gpu.py -x -q --timeout 240 --timeout-method thread -k "native or plan or ddp or sync or train" \
  > gpurun_out/wps/tests.log 2>&1
rc=$?; tail -4 gpurun_out/wps/tests.log; [ $rc -eq 0 ] || exit $rc
ab() {  # batch steps rounds
  for r in $(seq $3); do
    for v in 0 1; do
      RDP_WPREP_SIDE=$v timeout -k 10 300 python bench.py --batch $1 --steps $2 --warmup 8 --serve 0 --extras 0 \
        > gpurun_out/wps/b$1_$v.json 2>> gpurun_out/wps/bench.err || exit 1
      echo "b$1 wprepside=$v round $r $(python -c "import json;d=json.load(open('gpurun_out/wps/b$1_$v.json'));print(d['value'],d['ms_per_step'])")"
    done
  done
}
ab 4 60 3 || exit 1
ab 64 20 2 || exit 1
