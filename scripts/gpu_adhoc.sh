set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export RDP_NO_BUILD=1
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
timeout -k 10 300 python bench.py --impl eager --batch 64 --steps 10 --warmup 3 > gpurun_out/eager_b64.json 2> gpurun_out/eager_b64.err || { tail -20 gpurun_out/eager_b64.err; exit 1; }
cat gpurun_out/eager_b64.json
