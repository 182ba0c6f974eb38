#!/bin/bash
# GPU check: GPU tests (TESTS=..., default all), then the default bench; AB="ENV=v1 ENV=v2" adds an
# interleaved step A/B of those settings (E1=a,E2=b sets several; 2 rounds, bs 64 and bs 4; ABARGS: extra bench.py arguments,
# ABBATCH: batch sizes; SKIPTESTS=1: no pytest; NOBENCH=1: no default bench).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export RDP_NO_BUILD=1
if [ -z "$SKIPTESTS" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu.log
fi
if [ -n "$AB" ]; then
  for r in 1 2; do for b in ${ABBATCH:-64 4}; do for e in $AB; do
    st=$([ $b = 4 ] && echo 200 || echo 25)
    env ${e//,/ } timeout -k 10 200 python bench.py --batch $b --steps $st --warmup 5 --serve 0 --extras 0 $ABARGS > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/ab.json').read().splitlines()[-1]);print('$e bs$b r$r',d['value'],d['ms_per_step'])"
  done; done; done
fi
if [ -z "$NOBENCH" ]; then
  timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
  tail -1 gpurun_out/bench.json | cut -c1-600
fi
