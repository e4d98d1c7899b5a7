# round-4 A/B: the fused heavy-job variant (libafgpu_fused.so) -- genome tests, then the bench of
# both libraries
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-r04j}; mkdir -p $O
AF_GPU_LIB=libafgpu_fused.so timeout -k 10 300 python -u -m pytest tests/test_gpu_genome.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/genome.log 2>&1 || { tail -30 $O/genome.log; exit 1; }
tail -1 $O/genome.log
for lib in libafgpu_fused.so libafgpu.so; do
  AF_GPU_LIB=$lib timeout -k 10 240 python3 -u bench.py --no-cpu --steps 3 --warmup 1 > $O/b_$lib.log 2>&1 || { tail -5 $O/b_$lib.log; exit 1; }
  echo "$lib $(grep -o '"ms_per_step": [0-9.]*' $O/b_$lib.log) $(grep -o '"genome_bwa_s4_s5": [0-9.]*' $O/b_$lib.log)"
done
