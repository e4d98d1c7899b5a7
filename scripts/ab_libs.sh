# A/B of in-tree library builds on the configs[2] bench (LIBS = space-separated file names), alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-ablib}; mkdir -p $O
for k in 1 2; do for lib in ${LIBS:-libafgpu.so}; do
  AF_GPU_LIB=$lib timeout -k 10 200 python3 -u bench.py --no-cpu --steps 8 --warmup 2 > $O/${lib}_$k.log 2>&1 || exit 1
  grep '^{' $O/${lib}_$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', $k, d['value'], d['ms_per_step'], d['phases_ms']['s2'])"
done; done
