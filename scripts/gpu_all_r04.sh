# the whole GPU suite as the driver runs it, then smoke
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-all04}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/gpu_all.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR" $O/gpu_all.log | awk '{print $NF, $1}' | sort | uniq -c | sort -rn | head -3
tail -3 $O/gpu_all.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
echo "$(grep -o '"ms_per_step": [0-9.]*' $O/bench.log) $(grep -o '"genome_bwa_s4_s5": [0-9.]*' $O/bench.log) $(grep -o '"s6_clipped": [0-9.]*' $O/bench.log)"
