# Batch shape at configs[2] (50 M pairs, one GPU): ms per step by
# S2 batch size (bwa chunks) and batches in flight
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/n1sweep; mkdir -p $O
for cfg in "240 4" "188 4" "250 3" "167 3" "188 8"; do
  set -- $cfg
  timeout -k 10 200 python3 -u bench.py --no-cpu --steps 8 --warmup 2 --batch-chunks $1 --inflight $2 > $O/b$1_i$2.log 2>&1 || { echo "FAIL $cfg"; tail -5 $O/b$1_i$2.log; exit 1; }
  grep '^{' $O/b$1_i$2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1 $2', d['config']['pairs_per_batch'], d['config']['batches'], d['ms_per_step'], d['phases_ms']['s2'])"
done
