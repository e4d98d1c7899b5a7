# GPU check of the configs[2] path: the gpu tests, a reduced C3 bench, then the full one
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-c3a}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 && \
AF_DEBUG_DISCOVER=1 timeout -k 10 150 python -u bench.py --config c3 --genome-scale 0.05 --pairs 2000000 --steps 3 --warmup 1 --no-cpu > $O/small.log 2>&1 && \
timeout -k 10 400 python -u bench.py ${BENCH_ARGS:---no-cpu} > $O/full.log 2>&1
echo rc=$?
tail -3 $O/gpu_tests.log; grep -v amdgpu.ids $O/small.log | tail -8; tail -12 $O/full.log
