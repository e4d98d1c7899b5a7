# Batch shape at the configs[3] N = 8 per-rank size on one GPU (50 M / 8 pairs): ms per step by
# S2 batch size (bwa chunks) and batches in flight
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/n8sweep; mkdir -p $O
for cfg in "47 4" "63 3" "94 2" "32 6" "24 8" "188 1"; do
  set -- $cfg
  timeout -k 10 200 python3 -u bench.py --no-cpu --steps 8 --warmup 2 --pairs 6250000 --batch-chunks $1 --inflight $2 > $O/b$1_i$2.log 2>&1 || { echo "FAIL $cfg"; tail -5 $O/b$1_i$2.log; exit 1; }
  grep '^{' $O/b$1_i$2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1 $2', d['config']['pairs_per_batch'], d['config']['batches'], d['ms_per_step'], d['phases_ms']['s2'])"
done
