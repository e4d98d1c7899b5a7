# round-4: genome tests, then three bench runs (step-time spread)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-r04l}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_genome.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/genome.log 2>&1 || { tail -30 $O/genome.log; exit 1; }
tail -1 $O/genome.log
for k in 1 2 3; do
  timeout -k 10 200 python3 -u bench.py --no-cpu --steps 5 --warmup 2 > $O/b$k.log 2>&1 || { tail -5 $O/b$k.log; exit 1; }
  echo "run $k $(grep -o '"ms_per_step": [0-9.]*' $O/b$k.log) $(grep -o '"genome_bwa_s4_s5": [0-9.]*' $O/b$k.log)"
done
