#!/bin/bash
# Kernel traces of the final code: bs-64 step, bs-4 step, serving frames, transposed-decoder step (one thread: rocprofv3's kernel
# tracing crashes on frames submitted from several threads).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R"; mkdir -p gpurun_out/fin
export RDP_NO_BUILD=1 PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/fin/prof_train -o train --output-format csv -- python3 $R/bench.py --batch 64 --steps 4 --warmup 3 --serve 0 --extras 0 > $R/gpurun_out/fin/prof_train.log 2>&1 || { tail -20 $R/gpurun_out/fin/prof_train.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/fin/prof_bs4 -o bs4 --output-format csv -- python3 $R/bench.py --batch 4 --steps 20 --warmup 5 --serve 0 --extras 0 > $R/gpurun_out/fin/prof_bs4.log 2>&1 || { tail -20 $R/gpurun_out/fin/prof_bs4.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/fin/prof_serve -o serve --output-format csv -- python3 -m robotic_discovery_platform_amd.serve.bench_serve --frames 200 --warmup 20 --train-steps 200 --e2e 0 --multi 0 > $R/gpurun_out/fin/prof_serve.log 2>&1 || { tail -20 $R/gpurun_out/fin/prof_serve.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/fin/prof_tr -o tr --output-format csv -- python3 $R/bench.py --decoder transposed --batch 64 --steps 4 --warmup 3 --serve 0 --extras 0 > $R/gpurun_out/fin/prof_tr.log 2>&1 || { tail -20 $R/gpurun_out/fin/prof_tr.log; exit 1; }
echo prof_ok
