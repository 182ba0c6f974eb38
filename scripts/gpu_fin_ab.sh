#!/bin/bash
# BN finalize fused into the consumer launch (RDP_FUSE_FIN): kernel + whole-model GPU tests, interleaved
# step A/B at bs 4 / 64, and a bs-4 kernel trace with the fusion on.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R"; mkdir -p gpurun_out/fin
export RDP_NO_BUILD=1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_unet_native_gpu.py tests/test_ddp_native_gpu.py \
  tests/test_syncbn_native_gpu.py -x -q --timeout 240 --timeout-method thread -k "fused_into or bn_ or native or plan or ddp or sync" \
  > gpurun_out/fin/tests.log 2>&1
rc=$?; tail -4 gpurun_out/fin/tests.log; [ $rc -eq 0 ] || exit $rc
ab() {  # batch steps rounds
  for r in $(seq $3); do
    for v in 0 1; do
      RDP_FUSE_FIN=$v timeout -k 10 300 python bench.py --batch $1 --steps $2 --warmup 8 --serve 0 --extras 0 \
        > gpurun_out/fin/b$1_$v.json 2>> gpurun_out/fin/bench.err || exit 1
      echo "b$1 fusefin=$v round $r $(python -c "import json;d=json.load(open('gpurun_out/fin/b$1_$v.json'));print(d['value'],d['ms_per_step'])")"
    done
  done
}
ab 4 60 3 || exit 1
ab 64 20 2 || exit 1
export PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/fin/prof_bs4 -o bs4 --output-format csv -- python3 $R/bench.py --batch 4 --steps 20 --warmup 5 --serve 0 --extras 0 > $R/gpurun_out/fin/prof_bs4.log 2>&1 || { tail -20 $R/gpurun_out/fin/prof_bs4.log; exit 1; }
echo prof_ok
