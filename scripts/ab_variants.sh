# A/B of build variants (AF_GPU_LIB) on the configs[2] step; VARIANTS names the .so files
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/variants; mkdir -p $O
for v in ${VARIANTS:-libafgpu.so}; do
  AF_GPU_LIB=$v timeout -k 10 300 python -u bench.py --no-cpu --steps 8 > $O/b_$v.log 2>&1 || { echo "FAIL $v"; tail -20 $O/b_$v.log; exit 1; }
  grep '^{' $O/b_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phases_ms']; print('$v', d['value'], d['ms_per_step'], p['s2'], p['genome_placement'], d['counts_per_step']['queries_placed'], d['counts_per_step']['tails_placed'], d['counts_per_step']['anchored'])"
done
