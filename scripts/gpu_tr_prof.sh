#!/bin/bash
# side-stream re-layout test, transposed-decoder bench + kernel trace
set -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R"; mkdir -p gpurun_out/tr
export RDP_NO_BUILD=1
timeout -k 10 300 python -u -m pytest tests/test_unet_native_gpu.py -x -q --timeout 240 --timeout-method thread \
  -k "side_stream or plan" > gpurun_out/tr/tests.log 2>&1
rc=$?; tail -3 gpurun_out/tr/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --decoder transposed --steps 20 --warmup 5 --serve 0 --extras 0 > gpurun_out/tr/bench_tr.json 2> gpurun_out/tr/bench_tr.err || { tail -5 gpurun_out/tr/bench_tr.err; exit 1; }
cat gpurun_out/tr/bench_tr.json
export PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/tr/prof -o tr --output-format csv -- python3 $R/bench.py --decoder transposed --batch 64 --steps 4 --warmup 3 --serve 0 --extras 0 > $R/gpurun_out/tr/prof.log 2>&1 || { tail -20 $R/gpurun_out/tr/prof.log; exit 1; }
echo prof_ok
