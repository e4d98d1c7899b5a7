# round-end measurement set: every GPU test, smoke, then scripts/profile_c3.sh (bench line with the
# CPU baseline, kernel trace, K1 FETCH_SIZE / WRITE_SIZE passes) and the configs[1] bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-final}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
TAG=${TAG:-final} bash scripts/profile_c3.sh || exit 1
timeout -k 10 300 python -u bench.py --config c2 --no-cpu > $O/bench_c2.log 2>&1 || exit 1
grep '^{' $O/bench_c2.log | cut -c1-200
