# round-4: BLAT without the parts cap (GPU == oracle), the pipeline tables, a bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-r04b}; mkdir -p $O
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_blat.py tests/test_pipeline.py tests/test_gpu_s5s6.py > $O/gpu_blat.log 2>&1 || { tail -40 $O/gpu_blat.log; exit 1; }
tail -1 $O/gpu_blat.log
timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | cut -c1-300; grep -o '"phases_ms": {[^}]*}' $O/bench.log; grep -o '"counts_per_step": {[^}]*}' $O/bench.log
