# Per-rank proxy of the configs[3] strong-scaling points on one GPU: the step on 50 M / N pairs
# (N = 1, 2, 4, 8); predicted whole-job rate = 50 M / (per-rank step time), before the exchange
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-proxy}; mkdir -p $O
for n in 1 2 4 8; do
  p=$((50000000 / n))
  timeout -k 10 200 python3 -u bench.py --no-cpu --steps 8 --warmup 2 --pairs $p > $O/n$n.log 2>&1 || exit 1
  grep '^{' $O/n$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($n, d['config']['pairs_per_batch'], d['config']['batches'], d['ms_per_step'], round(50e6/(d['ms_per_step']*1e-3)/1e6,1), 'M pairs/s predicted', d['phases_ms']['s2'])"
done
