set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export RDP_NO_BUILD=1
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 500 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_train -o train --output-format csv -- python3 $R/bench.py --batch 64 --steps 4 --warmup 3 --serve 0 > $R/gpurun_out/prof_train.log 2>&1 || { tail -20 $R/gpurun_out/prof_train.log; exit 1; }
RDP_WGRAD_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_serial -o serial --output-format csv -- python3 $R/bench.py --batch 64 --steps 4 --warmup 3 --serve 0 > $R/gpurun_out/prof_serial.log 2>&1 || { tail -20 $R/gpurun_out/prof_serial.log; exit 1; }
