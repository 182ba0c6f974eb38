set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export RDP_NO_BUILD=1
run() {  # name, env..., args
  local n=$1; shift
  local e=(); while [[ $1 == *=* ]]; do e+=("$1"); shift; done
  env "${e[@]}" timeout -k 10 300 python bench.py --serve 0 "$@" > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err || { tail -20 gpurun_out/ab_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab_$n.json'));print('$n',d['value'],d['ms_per_step'],d['config']['hipgraph'])"
}
for r in 1 2; do
run t512_$r RDP_WGRAD_TAIL_BLOCKS=512 --steps 40
run t2048_$r RDP_WGRAD_TAIL_BLOCKS=2048 --steps 40
run t4096_$r RDP_WGRAD_TAIL_BLOCKS=4096 --steps 40
done
run b4t512 RDP_WGRAD_TAIL_BLOCKS=512 --steps 40 --batch 4
run b4t2048 RDP_WGRAD_TAIL_BLOCKS=2048 --steps 40 --batch 4
