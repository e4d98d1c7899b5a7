# round 6: k_blat's resident waves per CU (its persistent grid) against G1's residency in the
# genome phase (env knobs, no rebuild); default = k_blat's occupancy (24 per CU)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-knobs6}; mkdir -p $O
run() {
  env "$@" timeout -k 10 200 python3 -u bench.py --no-cpu --steps 6 --warmup 2 > $O/k.log 2>&1 || exit 1
  echo "$* $(grep -o '"ms_per_step": [0-9.]*' $O/k.log) $(grep -o '"genome_bwa_s4_s5": [0-9.]*' $O/k.log)"
}
run X=1
run AF_BLAT_WAVES_PER_CU=4
run AF_BLAT_WAVES_PER_CU=8
run AF_BLAT_WAVES_PER_CU=12
run AF_BLAT_WAVES_PER_CU=16
run X=2
