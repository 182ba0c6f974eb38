#!/bin/bash
# A/B: kernel tests on the new build, then conv microbench + bench for base (ab/_C_base.so) and new.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export RDP_NO_BUILD=1
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_kernels_gpu.py tests/test_unet_native_gpu.py} -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_ab.log; [ $rc -eq 0 ] || exit $rc
fi
for round in 1 2; do
for v in base new; do
  if [ $v = base ]; then export RDP_NATIVE_SO=$GRAFT_REPO_ROOT/ab/_C_base.so; else unset RDP_NATIVE_SO; fi
  if [ -n "$MICRO" ]; then
    timeout -k 10 300 python scripts/conv_microbench.py $MICRO --out gpurun_out/micro_${v}_$round.json > gpurun_out/micro_${v}_$round.log 2>&1 || { tail -20 gpurun_out/micro_${v}_$round.log; exit 1; }
  fi
  for b in ${BATCHES:-64}; do
    timeout -k 10 300 python bench.py --batch $b --steps 20 --warmup 5 --serve 0 --extras 0 > gpurun_out/ab_${v}_b${b}_$round.json 2> gpurun_out/ab_${v}_b${b}_$round.err || { tail -20 gpurun_out/ab_${v}_b${b}_$round.err; exit 1; }
    echo "$v b$b round$round $(python3 -c "import json;d=json.load(open('gpurun_out/ab_${v}_b${b}_$round.json'));print(d['value'], d['ms_per_step'])")"
  done
done
done
