# bench step time of several in-tree library builds (name suffixes as arguments; base = libafgpu.so)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
  if [ "$v" = base ]; then lib=libafgpu.so; else lib=libafgpu_$v.so; fi
  AF_GPU_LIB=$lib timeout -k 10 200 python3 bench.py --no-cpu --steps 20 2>/dev/null | tail -1 | \
    python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['ms_per_step'], d['kernels_ms'])" || exit 1
done
