# k_blat's launch bound (AF_BLAT_WPS waves per SIMD: the VGPR budget vs spills) on the configs[2]
# step: in-tree variants libafgpu_w<N>.so (make OUT=../libafgpu_w<N>.so EXTRA=-DAF_BLAT_WPS=<N>)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-wps}; mkdir -p $O
for w in ${WPS:-4 5 6 8}; do
  lib=libafgpu_w$w.so; [ "$w" = 6 ] && lib=libafgpu.so
  AF_GPU_LIB=$lib timeout -k 10 200 python3 -u bench.py --no-cpu --steps 5 --warmup 2 > $O/w$w.log 2>&1 || exit 1
  echo "wps $w $(grep -o '"ms_per_step": [0-9.]*' $O/w$w.log) $(grep -o '"genome_bwa_s4_s5": [0-9.]*' $O/w$w.log)"
done
