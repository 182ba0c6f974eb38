#!/bin/bash
# Torch-eager (MIOpen) baseline of the reference training step on 1x MI355X.
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
python -c "import torch;print(torch.cuda.get_device_name(0))" || exit 1
for b in 4 16 32 64; do
  timeout -k 10 300 python bench.py --impl eager --batch $b --steps 10 --warmup 3 > gpurun_out/eager_b$b.json 2> gpurun_out/eager_b$b.err || exit 1
  cat gpurun_out/eager_b$b.json
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_eager -o eager --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --impl eager --batch 32 --steps 3 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_eager.log 2>&1
echo prof_rc=$?
