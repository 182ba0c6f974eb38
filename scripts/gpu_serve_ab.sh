#!/bin/bash
# Serving engine A/B of an env knob, interleaved on one box: KNOB=NAME A=value B=value (ROUNDS, default 2).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/sab
export RDP_NO_BUILD=1
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in "$A" "$B"; do
    env $KNOB=$v timeout -k 10 240 python -m robotic_discovery_platform_amd.serve.bench_serve --frames 400 --warmup 40 --train-steps 20 ${SERVE_ARGS:---e2e 0 --multi 0} > gpurun_out/sab/r${r}_$v.log 2>&1 || { tail -20 gpurun_out/sab/r${r}_$v.log; exit 1; }
    echo "round $r $KNOB=$v: $(grep -o '"serve_engine_fps.*' gpurun_out/sab/r${r}_$v.log | tail -1)"
  done
done
