# configs[2] measurement set (TAG names the output dir): the default bench line (with the CPU
# baseline), a rocprofv3 kernel trace of the bench, and FETCH_SIZE / WRITE_SIZE counter passes
# on K1 (k_seed_stream) in runs of their own
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-c3m}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py ${BENCH_ARGS:-} > $O/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu > $O/kt.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_seed_stream --output-format csv -d $O/fetch -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu > $O/fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_seed_stream --output-format csv -d $O/write -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu > $O/write.log 2>&1
echo rc=$?
grep '^{' $O/bench.log | cut -c1-400
f=$(find $O/kt -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -d, -f1-8 "$f" | head -16
