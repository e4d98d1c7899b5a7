# round-4: BLAT spill pool (GPU == oracle's full row lists), BLAT / pipeline / dist tables, bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-r04c}; mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_blat.py tests/test_pipeline.py tests/test_gpu_s5s6.py tests/test_gpu_dist.py > $O/gpu_blat.log 2>&1 || { tail -40 $O/gpu_blat.log; exit 1; }
tail -1 $O/gpu_blat.log
timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | cut -c1-200; grep -o '"phases_ms": {[^}]*}' $O/bench.log; grep -o '"counts_per_step": {[^}]*}' $O/bench.log
