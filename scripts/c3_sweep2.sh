# configs[2] bench sweep over S2 batch size and batches in flight (TAG names the output dir)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-sw2}; mkdir -p $O
for bc in 125 250; do for inf in 2 3 4 6; do
  timeout -k 10 200 python3 -u bench.py --no-cpu --steps 5 --warmup 1 --batch-chunks $bc --inflight $inf > $O/b_${bc}_${inf}.log 2>&1 || exit 1
  grep '^{' $O/b_${bc}_${inf}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($bc, $inf, d['value'], d['ms_per_step'], d['phases_ms']['s2'], d['phases_ms']['genome_placement'], d['roofline']['frac'])"
done; done
