# configs[2] GPU tests + a rocprofv3 kernel trace of the C3 bench (TAG names the output dir)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-c3p}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_c3.py tests/test_gpu_align.py -k "${TESTS:-c3 or world or discovery or tandem}" -x -v --timeout 500 --timeout-method thread > $O/tests.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 4 --warmup 1 --no-cpu > $O/bench_prof.log 2>&1
echo rc=$?
tail -12 $O/tests.log; tail -2 $O/bench_prof.log | cut -c1-600
f=$(find $O/kt -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -d, -f1-8 "$f" | head -25
