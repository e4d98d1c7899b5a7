# every gpu test + smoke + the default bench line + the c2 bench line (TAG names the output dir)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-ga}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > $O/bench.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c2 --no-cpu > $O/bench_c2.log 2>&1
echo rc=$?
grep -E "FAILED|ERROR" $O/gpu_tests.log | head -5; tail -2 $O/gpu_tests.log; tail -1 $O/smoke.log
grep '^{' $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C3', d['value'], d['ms_per_step'], d['phases_ms'], d['roofline']['frac'], d.get('cpu_baseline',{}).get('value'), d['counts_per_step'])"
grep '^{' $O/bench_c2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C2', d['value'], d['ms_per_step'], d['partner_placement'], d['s2_only'])"
