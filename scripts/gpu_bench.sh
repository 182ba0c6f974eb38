#!/bin/bash
# Native bench at several per-GPU batches + a rocprofv3 kernel-time profile of one config.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export RDP_NO_BUILD=1
for b in ${BATCHES:-4 32}; do
  timeout -k 10 300 python bench.py --impl native --batch $b --steps ${STEPS:-20} --warmup 5 > gpurun_out/native_b$b.json 2> gpurun_out/native_b$b.err || { tail -20 gpurun_out/native_b$b.err; exit 1; }
  cat gpurun_out/native_b$b.json
done
if [ -n "$PROF" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_native -o native --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --impl native --batch $PROF --steps 3 --warmup 2 --graph 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_native.log 2>&1
  echo prof_rc=$?
fi
