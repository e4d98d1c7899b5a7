# K1 change check: every GPU test, the default bench line, and a kernel trace of the bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-k1c}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 400 python -u bench.py --no-cpu > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['phases_ms']['s2'], d['roofline']['frac'], d['kernels_ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu > $O/kt.log 2>&1 || exit 1
f=$(find $O/kt -name "*kernel_stats.csv" | head -1); grep k_seed_stream "$f" | awk -F'",' '{print $2}'
