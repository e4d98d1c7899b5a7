# all gpu-marked tests + smoke (TAG names the output dir)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-gt}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread ${PYTEST_ARGS:-} > $O/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo rc=$?
grep -E "PASSED|FAILED|ERROR" $O/gpu_tests.log | tail -5; tail -3 $O/gpu_tests.log; tail -1 $O/smoke.log
