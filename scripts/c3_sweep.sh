# configs[2] bench over S2 batch sizes and batches in flight (one line per setting)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-c3s}; mkdir -p $O
for cfg in ${CFGS:-"30 8" "60 8" "120 4" "30 12" "60 4"}; do
  set -- $cfg
  timeout -k 10 200 python -u bench.py --no-cpu --steps 6 --warmup 1 --batch-chunks $1 --inflight $2 > $O/b_$1_$2.log 2>&1 || exit $?
  grep '^{' $O/b_$1_$2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1 $2', d['value'], d['ms_per_step'], d['phases_ms']['s2'], d['phases_ms']['genome_placement'], d['roofline']['frac'], d['kernels_ms']['seed_filter_per_launch'])"
done
