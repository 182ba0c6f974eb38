set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export RDP_NO_BUILD=1
R=$GRAFT_REPO_ROOT
run() {  # name, env..., args
  local n=$1; shift
  local e=(); while [[ $1 == *=* ]]; do e+=("$1"); shift; done
  env "${e[@]}" timeout -k 10 300 python bench.py --serve 0 "$@" > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err || { tail -20 gpurun_out/ab_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab_$n.json'));print('$n',d['value'],d['ms_per_step'],d['config']['hipgraph'])"
}
run b64_prio RDP_MAIN_PRIO=1 --batch 64 --steps 40
run b64_noprio RDP_MAIN_PRIO=0 --batch 64 --steps 40
run b64_prio2 RDP_MAIN_PRIO=1 --batch 64 --steps 40
run b64_g1 RDP_MAIN_PRIO=1 --batch 64 --steps 40 --graph 1
run b32_g0 RDP_MAIN_PRIO=1 --batch 32 --steps 40 --graph 0
run b32_g1 RDP_MAIN_PRIO=1 --batch 32 --steps 40 --graph 1
run b16_g0 RDP_MAIN_PRIO=1 --batch 16 --steps 40 --graph 0
run b16_g1 RDP_MAIN_PRIO=1 --batch 16 --steps 40 --graph 1
run b4_g0 RDP_MAIN_PRIO=1 --batch 4 --steps 40 --graph 0
run b4_g1 RDP_MAIN_PRIO=1 --batch 4 --steps 40 --graph 1
