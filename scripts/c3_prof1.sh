# rocprofv3 kernel trace of the C3 bench with one batch in flight (true per-kernel times)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-c3p1}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu ${BENCH_ARGS:---inflight 1} > $O/bench_prof.log 2>&1
echo rc=$?
grep '^{' $O/bench_prof.log | cut -c1-300
