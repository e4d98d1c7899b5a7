# A/B of two library builds at 2x100 and 2x150 (bench step times), interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do
  for v in "$@"; do
    if [ "$v" = base ]; then lib=libafgpu.so; else lib=libafgpu_$v.so; fi
    for L in 100 150; do
      AF_GPU_LIB=$lib timeout -k 10 200 python3 bench.py --no-cpu --steps 20 --read-len $L 2>/dev/null | tail -1 | \
        python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', $L, d['ms_per_step'], d['kernels_ms'])" || exit 1
    done
  done
done
