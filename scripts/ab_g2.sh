# A/B: S4 / S5 as two concurrent genome calls (AF_S4_SPLIT=1) or one (0), and the heavy-read
# threshold of G2 (AF_G_HEAVY_CHAINS); parity of the split step first
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-abg2b}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_c3.py -k reduced tests/test_pipeline.py > $O/par.log 2>&1 || { tail -30 $O/par.log; exit 1; }
echo "parity: $(tail -1 $O/par.log)"
for cfg in ${CFGS:-"0 16" "1 16" "1 4" "1 1"}; do
  set -- $cfg
  AF_S4_SPLIT=$1 AF_G_HEAVY_CHAINS=$2 timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu > $O/bench_s$1_h$2.log 2>&1 || { tail -20 $O/bench_s$1_h$2.log; exit 1; }
  echo "split $1 heavy $2: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_s$1_h$2.log) $(grep -o '"genome_bwa_s4_s5": [0-9.]*' $O/bench_s$1_h$2.log)"
done
