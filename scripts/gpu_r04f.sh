# G2 region boxes in LDS + BLAT scratch sized per search: genome / BLAT parity, the single-cell
# configs[4] rank test (many tile contexts), a bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-r04f}; mkdir -p $O
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_genome.py tests/test_gpu_blat.py tests/test_gpu_configs.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
echo "$(grep -o '"ms_per_step": [0-9.]*' $O/bench.log) $(grep -o '"genome_bwa_s4_s5": [0-9.]*' $O/bench.log) $(grep -o '"hbm_in_use_gib": [0-9.]*' $O/bench.log)"
