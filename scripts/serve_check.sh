set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export RDP_NO_BUILD=1
timeout -k 10 400 python -u -m pytest tests/test_serve_gpu.py tests/test_serve_replicas_gpu.py tests/test_train_serve_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_serve.log 2>&1 || { tail -30 gpurun_out/pytest_serve.log; exit 1; }
tail -3 gpurun_out/pytest_serve.log
timeout -k 10 400 python scripts/serve_e2e_ab.py --switch 0 --streams ${STREAMS:-1,4,8} --procs ${PROCS:-2:4,4:4,4:8,8:8} > gpurun_out/e2e_ab2.jsonl 2> gpurun_out/e2e_ab2.err
