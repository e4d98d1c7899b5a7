# K1 loads-in-flight sweep at configs[2] (HBM-resident reads, distinct ranges): bench per build variant
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/k1depth; mkdir -p $O
for v in libafgpu.so libafgpu_d3.so libafgpu_d4.so libafgpu_d4nt.so; do
  AF_GPU_LIB=$v timeout -k 10 300 python -u bench.py --no-cpu --steps 6 > $O/bench_$v.log 2>&1 || { echo "FAIL $v"; tail -20 $O/bench_$v.log; exit 1; }
  grep '^{' $O/bench_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'], d['phases_ms']['s2'], d['roofline']['frac'], d['kernels_ms'])"
done
