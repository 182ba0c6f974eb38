set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export RDP_NO_BUILD=1
R=$GRAFT_REPO_ROOT; export PYTHONPATH=$R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_tr
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_tr -o tr --output-format csv -- \
  python3 $R/bench.py --batch 64 --steps 4 --warmup 3 --serve 0 --decoder transposed > $R/gpurun_out/prof_tr.log 2>&1 || { tail -20 $R/gpurun_out/prof_tr.log; exit 1; }
grep '"metric"' $R/gpurun_out/prof_tr.log
