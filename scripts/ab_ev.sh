set -o pipefail
cd "$GRAFT_REPO_ROOT"; export RDP_NO_BUILD=1
for r in 1 2; do for ab in 0 1 2; do for b in 4 64; do
RDP_AB_EVFLAGS=$ab timeout -k 10 200 python bench.py --batch $b --steps 30 --warmup 5 --serve 0 --extras 0 > gpurun_out/ev_${ab}_b${b}_$r.json 2> gpurun_out/abev.err || exit 1
done; done; done
bash scripts/gpu_evidence2.sh
