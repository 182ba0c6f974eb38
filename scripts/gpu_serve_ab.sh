#!/bin/bash
# A/B of the serving engine (no e2e): base = ab/_C_base.so, new = the in-tree build; kernel tests first.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export RDP_NO_BUILD=1
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_kernels_gpu.py} -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_sab.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_sab.log; [ $rc -eq 0 ] || exit $rc
fi
for round in 1 2; do
for v in base new; do
  if [ $v = base ]; then export RDP_NATIVE_SO=$GRAFT_REPO_ROOT/ab/_C_base.so; else unset RDP_NATIVE_SO; fi
  timeout -k 10 300 python -m robotic_discovery_platform_amd.serve.bench_serve --frames ${FRAMES:-400} --warmup 40 --train-steps 20 --e2e 0 > gpurun_out/sab_${v}_$round.json 2> gpurun_out/sab_${v}_$round.err || { tail -20 gpurun_out/sab_${v}_$round.err; exit 1; }
  echo "$v round$round $(python3 -c "import json;d=json.load(open('gpurun_out/sab_${v}_$round.json'));e=d.get('engine',d);print({k:v for k,v in e.items() if not isinstance(v,(dict,list))})")"
done
done
