set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export RDP_NO_BUILD=1
R=$GRAFT_REPO_ROOT; export PYTHONPATH=$R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "bnred or ring" > gpurun_out/t_k.log 2>&1 || { tail -30 gpurun_out/t_k.log; exit 1; }
tail -1 gpurun_out/t_k.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_unet_native_gpu.py > gpurun_out/t_u.log 2>&1 || { tail -30 gpurun_out/t_u.log; exit 1; }
tail -1 gpurun_out/t_u.log
run() {  # name, env..., args
  local n=$1; shift
  local e=(); while [[ $1 == *=* ]]; do e+=("$1"); shift; done
  env "${e[@]}" timeout -k 10 300 python bench.py --serve 0 "$@" > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err || { tail -20 gpurun_out/ab_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab_$n.json'));print('$n',d['value'],d['ms_per_step'])"
}
for r in 1 2; do
run on_$r RDP_DGRAD_BNRED=1 --steps 40
run off_$r RDP_DGRAD_BNRED=0 --steps 40
done
run b4on RDP_DGRAD_BNRED=1 --steps 40 --batch 4
run b4off RDP_DGRAD_BNRED=0 --steps 40 --batch 4
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
rm -rf $R/gpurun_out/prof_bn$v
RDP_DGRAD_BNRED=$v RDP_WGRAD_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_bn$v -o bn --output-format csv -- \
  python3 $R/bench.py --batch 64 --steps 4 --warmup 3 --serve 0 > $R/gpurun_out/prof_bn$v.log 2>&1 || { tail -20 $R/gpurun_out/prof_bn$v.log; exit 1; }
done
