# G1 heavy-read handoff: parity of the wave path, then bench lines: the previous build
# (libafgpu_v0.so) and the current one at several handoff thresholds (AF_G1_HEAVY_EXT)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-abg1}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_genome.py > $O/par.log 2>&1 || { tail -30 $O/par.log; exit 1; }
echo "parity: $(tail -1 $O/par.log)"
[ -n "$SKIP_V0" ] || AF_GPU_LIB=libafgpu_v0.so timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu > $O/bench_v0.log 2>&1 || { tail -20 $O/bench_v0.log; exit 1; }
[ -n "$SKIP_V0" ] || echo "v0 $(grep -o '"ms_per_step": [0-9.]*' $O/bench_v0.log) $(grep -o '"genome_bwa_s4_s5": [0-9.]*' $O/bench_v0.log)"
for t in ${THRESHOLDS:-0 1024 2048 4096}; do
  AF_G1_HEAVY_EXT=$t timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu > $O/bench_t$t.log 2>&1 || { tail -20 $O/bench_t$t.log; exit 1; }
  echo "t$t $(grep -o '"ms_per_step": [0-9.]*' $O/bench_t$t.log) $(grep -o '"genome_bwa_s4_s5": [0-9.]*' $O/bench_t$t.log)"
done
