# K1 timing of several in-tree library builds (name suffixes as arguments), one probe each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
  if [ "$v" = base ]; then lib=libafgpu.so; else lib=libafgpu_$v.so; fi
  AF_GPU_LIB=$lib timeout -k 10 120 python3 scripts/k1_probe.py 2>&1 | grep k1 | sed "s/^/$v /" || exit 1
done
