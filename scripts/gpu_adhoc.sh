set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export RDP_NO_BUILD=1
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_unet_native_gpu.py tests/test_race_screens_gpu.py > gpurun_out/t_u.log 2>&1 || { tail -30 gpurun_out/t_u.log; exit 1; }
tail -1 gpurun_out/t_u.log
run() {  # name, env..., args
  local n=$1; shift
  local e=(); while [[ $1 == *=* ]]; do e+=("$1"); shift; done
  env "${e[@]}" timeout -k 10 300 python bench.py --serve 0 "$@" > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err || { tail -20 gpurun_out/ab_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab_$n.json'));print('$n',d['value'],d['ms_per_step'],d['config']['hipgraph'])"
}
run b64 --steps 40
run b4 --steps 40 --batch 4
cd /tmp && export TMPDIR=/tmp
RDP_WGRAD_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_serial -o serial --output-format csv -- python3 $R/bench.py --batch 64 --steps 4 --warmup 3 --serve 0 > $R/gpurun_out/prof_serial.log 2>&1 || { tail -20 $R/gpurun_out/prof_serial.log; exit 1; }
