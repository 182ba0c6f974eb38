#!/bin/bash
# Launch-plan event binding (RDP_PLAN_BIND): plan replay tests, interleaved step A/B at bs 4 / 64, and a
# bs-4 kernel trace with binding on.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R"; mkdir -p gpurun_out/bind
export RDP_NO_BUILD=1
timeout -k 10 400 python -u -m pytest tests/test_unet_native_gpu.py tests/test_kernels_gpu.py -x -q --timeout 200 \
  --timeout-method thread -k "plan or replay or pingpong_splitk or graph" > gpurun_out/bind/tests.log 2>&1
rc=$?; tail -4 gpurun_out/bind/tests.log; [ $rc -eq 0 ] || exit $rc
ab() {  # batch steps tag
  for r in 1 2 3; do
    for v in 0 1; do
      RDP_PLAN_BIND=$v timeout -k 10 300 python bench.py --batch $1 --steps $2 --warmup 8 --serve 0 --extras 0 \
        > gpurun_out/bind/b$1_$v.json 2>> gpurun_out/bind/bench.err || exit 1
      echo "b$1 bind=$v round $r $(python -c "import json;d=json.load(open('gpurun_out/bind/b$1_$v.json'));print(d['value'],d['ms_per_step'])")"
    done
  done
}
ab 4 60 || exit 1
ab 64 20 || exit 1
export PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/bind/prof_bs4 -o bs4 --output-format csv -- python3 $R/bench.py --batch 4 --steps 20 --warmup 5 --serve 0 --extras 0 > $R/gpurun_out/bind/prof_bs4.log 2>&1 || { tail -20 $R/gpurun_out/bind/prof_bs4.log; exit 1; }
echo prof_ok
