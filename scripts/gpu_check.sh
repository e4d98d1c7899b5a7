# full GPU check: every gpu-marked test, smoke(), the default bench line (TAG names the output dir)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-r1}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 400 python bench.py > $O/bench.log 2>&1
echo rc=$?
tail -3 $O/gpu_tests.log; cat $O/smoke.log; tail -1 $O/bench.log
