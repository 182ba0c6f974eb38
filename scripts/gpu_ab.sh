set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export RDP_NO_BUILD=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "ring" -x -q --timeout 120 --timeout-method thread > gpurun_out/ring2_test.log 2>&1 || { tail -30 gpurun_out/ring2_test.log; exit 1; }
tail -2 gpurun_out/ring2_test.log
timeout -k 10 300 python scripts/conv_microbench.py --batch 64 --shapes 9,10,8 --variants 0,3,256,14 --out gpurun_out/micro_ring2.json > gpurun_out/micro_ring2.log 2>&1 || { tail -20 gpurun_out/micro_ring2.log; exit 1; }
tail -8 gpurun_out/micro_ring2.log
for r in 1 2; do for v in 0 1; do
RDP_RING2=$v timeout -k 10 200 python bench.py --serve 0 --extras 0 > gpurun_out/b_r2.json 2>gpurun_out/b_r2.err || { tail -20 gpurun_out/b_r2.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/b_r2.json').read().splitlines()[-1]);print('RDP_RING2=$v r$r',d['value'],d['ms_per_step'])"
done; done
