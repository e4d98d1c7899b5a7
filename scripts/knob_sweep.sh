# round-4: the genome calls' scheduling knobs on the configs[2] step (env, no rebuild):
# AF_G_HEAVY_CHAINS (kept chains that defer a read to the chain jobs) and AF_G2_FIRST_OCC
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-knobs}; mkdir -p $O
run() {
  env "$@" timeout -k 10 200 python3 -u bench.py --no-cpu --steps 4 --warmup 1 > $O/k.log 2>&1 || exit 1
  echo "$* $(grep -o '"ms_per_step": [0-9.]*' $O/k.log) $(grep -o '"genome_bwa_s4_s5": [0-9.]*' $O/k.log)"
}
run AF_G_HEAVY_CHAINS=16
run AF_G_HEAVY_CHAINS=8
run AF_G_HEAVY_CHAINS=32
run AF_G_HEAVY_CHAINS=64
run AF_G2_FIRST_OCC=0
run AF_G2_FIRST_OCC=32
run AF_G2_FIRST_OCC=512
