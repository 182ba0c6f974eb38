set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export RDP_NO_BUILD=1
run() {  # name, env..., args
  local n=$1; shift
  local e=(); while [[ $1 == *=* ]]; do e+=("$1"); shift; done
  env "${e[@]}" timeout -k 10 300 python bench.py --serve 0 "$@" > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err || { tail -20 gpurun_out/ab_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab_$n.json'));print('$n',d['value'],d['ms_per_step'],d['config']['hipgraph'])"
}
for r in 1 2; do
run w768_$r RDP_WGRAD_BLOCKS=768 --steps 40
run w2048_$r RDP_WGRAD_BLOCKS=2048 --steps 40
run w512_$r RDP_WGRAD_BLOCKS=512 --steps 40
run w1024_$r RDP_WGRAD_BLOCKS=1024 --steps 40
done
