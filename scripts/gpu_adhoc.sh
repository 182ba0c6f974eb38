set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export RDP_NO_BUILD=1
run() {  # name, env..., args
  local n=$1; shift
  local e=(); while [[ $1 == *=* ]]; do e+=("$1"); shift; done
  env "${e[@]}" timeout -k 10 300 python bench.py --serve 0 "$@" > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err || { tail -20 gpurun_out/ab_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab_$n.json'));print('$n',d['value'],d['ms_per_step'],d['config']['hipgraph'])"
}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_unet_native_gpu.py tests/test_ddp_native_gpu.py tests/test_kernels_gpu.py -k "adam or native or ddp" > gpurun_out/t_u.log 2>&1 || { tail -30 gpurun_out/t_u.log; exit 1; }
tail -1 gpurun_out/t_u.log
for r in 1 2; do
run ao0_$r RDP_ADAM_OVERLAP=0 --steps 40
run ao1_$r RDP_ADAM_OVERLAP=1 --steps 40
done
run b4ao0 RDP_ADAM_OVERLAP=0 --steps 40 --batch 4
run b4ao1 RDP_ADAM_OVERLAP=1 --steps 40 --batch 4
