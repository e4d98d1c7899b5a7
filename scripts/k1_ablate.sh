# K1 ablation: the product kernel (0) against the stream-only build (1) = the memory floor
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for v in 0 1 4; do
  if [ "$v" = 0 ]; then lib=libafgpu.so; else lib=libafgpu_abl$v.so; fi
  AF_GPU_LIB=$lib timeout -k 10 120 python3 scripts/k1_probe.py 2>&1 | grep k1 | sed "s/^/abl$v /" || exit 1
done
