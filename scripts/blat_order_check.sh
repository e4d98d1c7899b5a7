set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/ord; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_blat.py tests/test_gpu_c3.py tests/test_pipeline.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || exit 1
for n in 1 8; do
  p=$((50000000 / n))
  timeout -k 10 200 python3 -u bench.py --no-cpu --steps 8 --warmup 2 --pairs $p > $O/n$n.log 2>&1 || exit 1
  grep '^{' $O/n$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($n, d['ms_per_step'], round(50e6/(d['ms_per_step']*1e-3)/1e6,1), d['phases_ms'])"
done
tail -1 $O/t.log
