set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r1b
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r1b/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r1b/smoke.log 2>&1 && \
timeout -k 10 400 python bench.py > gpurun_out/r1b/bench.log 2>&1
echo rc=$?
tail -3 gpurun_out/r1b/gpu_tests.log; cat gpurun_out/r1b/smoke.log; tail -2 gpurun_out/r1b/bench.log
