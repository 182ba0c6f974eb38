#!/bin/bash
# Does the GPU test suite leave processes behind that slow the bench run after it (the reference-batch
# number is host-sensitive)? Full suite, then the process list, then bench.py without serving.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export RDP_NO_BUILD=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/lo_pytest.log 2>&1
rc=$?
tail -2 gpurun_out/lo_pytest.log
[ $rc -ne 0 ] && exit $rc
ps -eo pid,ppid,pcpu,etime,args --sort=-pcpu > gpurun_out/lo_ps.txt 2>&1 || true
head -25 gpurun_out/lo_ps.txt
timeout -k 10 300 python bench.py --serve 0 > gpurun_out/lo_bench.json 2> gpurun_out/lo_bench.err || exit 1
python -c "import json; d=json.loads(open('gpurun_out/lo_bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ref_batch_imgs_per_s'], d['ref_batch_ms_per_step'], d['train_model_imgs_per_s'])"
ps -eo pid,ppid,pcpu,etime,args --sort=-pcpu | head -12
