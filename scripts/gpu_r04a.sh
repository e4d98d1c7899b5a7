# round-4 iteration: genome parity tests (incl. the 2 % world vs the oracle's own index and genome
# calls), the per-read genome profile, a short bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-r04a}; mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_genome.py tests/test_gpu_s5s6.py tests/test_pipeline.py > $O/gpu_genome.log 2>&1 || { tail -40 $O/gpu_genome.log; exit 1; }
tail -1 $O/gpu_genome.log
timeout -k 10 400 $T tests/test_gpu_c3.py -k reduced > $O/gpu_reduced.log 2>&1 || { tail -40 $O/gpu_reduced.log; exit 1; }
tail -1 $O/gpu_reduced.log
timeout -k 10 300 python3 -u scripts/g_prof.py > $O/gprof.log 2>&1 || { tail -30 $O/gprof.log; exit 1; }
grep -v "^ " $O/gprof.log | tail -3; grep -E "G1 cycles|G2 cycles|shares|makespan" $O/gprof.log
timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | cut -c1-300; grep -o '"phases_ms": {[^}]*}' $O/bench.log
