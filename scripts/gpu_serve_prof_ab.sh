#!/bin/bash
# Serving-frame kernel timelines (rocprofv3 --kernel-trace) for base (ab/_C_base.so) and new builds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export RDP_NO_BUILD=1
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS:-base new}; do
  if [ $v = base ]; then export RDP_NATIVE_SO=$R/ab/_C_base.so; else unset RDP_NATIVE_SO; fi
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/sprof_$v -o sp --output-format csv -- python3 -m robotic_discovery_platform_amd.serve.bench_serve --frames 100 --warmup 20 --train-steps ${TRAIN_STEPS:-5} --e2e 0 > $R/gpurun_out/sprof_$v.log 2>&1 || { tail -20 $R/gpurun_out/sprof_$v.log; exit 1; }
  tr=$(ls $R/gpurun_out/sprof_$v/*/sp_kernel_trace.csv 2>/dev/null || find $R/gpurun_out/sprof_$v -name 'sp_kernel_trace.csv' | head -1)
  python3 $R/scripts/serve_frame.py $tr > $R/gpurun_out/sprof_$v.txt
  echo "== $v"; tail -3 $R/gpurun_out/sprof_$v.txt
done
