# One GPU iteration: the named pytest files (TESTS, default: the S5/S6 + BLAT + c3 reduced set),
# then a short bench line with its phases (STEPS steps), each step under its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-check}; mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
TESTS=${TESTS:-"tests/test_gpu_s5s6.py tests/test_gpu_blat.py"}
if [ "$TESTS" != "none" ]; then
  timeout -k 10 900 $T $TESTS ${KSEL:+-k "$KSEL"} > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
timeout -k 10 300 python3 -u bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | cut -c1-240; grep -o '"phases_ms": {[^}]*}' $O/bench.log
