set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export RDP_NO_BUILD=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_unet_native_gpu.py -k "transpose or decoder or native" > gpurun_out/t_tr.log 2>&1 || { tail -30 gpurun_out/t_tr.log; exit 1; }
tail -1 gpurun_out/t_tr.log
for a in "--decoder transposed" "--decoder transposed --batch 4" "--decoder bilinear"; do
timeout -k 10 300 python bench.py --serve 0 --steps 30 $a > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$a',d['value'],d['ms_per_step'])"
done
