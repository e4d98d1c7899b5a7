# A/B of the post-S2 schedule (S4/S5 placement beside the S6 BLAT)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r02_post; mkdir -p $O
run() { tag=$1; shift; timeout -k 10 300 python -u bench.py --no-cpu --steps 8 "$@" > $O/bench_$tag.log 2>&1 || { echo "BENCHFAIL $tag"; tail -20 $O/bench_$tag.log; exit 1; }
  grep '^{' $O/bench_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phases_ms']; print('$tag', d['value'], d['ms_per_step'], p['s2'], p['s3_partition'], p['genome_placement'])"; }
run base
AF_BLAT_WAVES_PER_CU=8 run bw8
AF_BLAT_WAVES_PER_CU=12 run bw12
AF_PLACE_FIRST=1 run pf
AF_PLACE_FIRST=1 AF_BLAT_WAVES_PER_CU=12 run pf_bw12
