# G2 A/B: the heavy-read threshold (AF_G_HEAVY_CHAINS: reads with this many kept chains extend
# them one job per chain), bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-abg2b}; mkdir -p $O
for t in ${THRESHOLDS:-1 4 8 16}; do
  AF_G_HEAVY_CHAINS=$t timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu > $O/bench_h$t.log 2>&1 || { tail -20 $O/bench_h$t.log; exit 1; }
  echo "h$t $(grep -o '"ms_per_step": [0-9.]*' $O/bench_h$t.log) $(grep -o '"genome_bwa_s4_s5": [0-9.]*' $O/bench_h$t.log)"
done
