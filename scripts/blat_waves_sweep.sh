# k_blat resident waves per CU (AF_BLAT_WAVES_PER_CU) on the configs[2] step: the scratch working
# set (waves x ~60 KB of hit keys) against latency hiding
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/bw; mkdir -p $O
for w in 0 8 12 16; do
  AF_BLAT_WAVES_PER_CU=$w timeout -k 10 200 python3 -u bench.py --no-cpu --steps 6 --warmup 2 > $O/w$w.log 2>&1 || exit 1
  grep '^{' $O/w$w.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phases_ms']; print($w, d['ms_per_step'], round(p['s3_partition']+p['gather_queries']+p['genome_placement'],2))"
done
