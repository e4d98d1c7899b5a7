# Bench lines under environment variants: KNOBS="A=1 B=2;A=2" (';' separates runs), then a kernel
# trace + step timeline of the first variant when TRACE=1.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-knobs}; mkdir -p $O
export TMPDIR=/tmp
IFS=';' read -ra V <<< "${KNOBS:-}"
i=0
for v in "${V[@]}"; do
  env $v timeout -k 10 300 python3 -u bench.py --steps ${STEPS:-4} --warmup 1 --no-cpu > $O/bench_$i.log 2>&1 || { echo "[$v] failed"; tail -20 $O/bench_$i.log; exit 1; }
  echo "[$v] $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$i.log) $(grep -o '"genome_bwa_s4_s5": [0-9.]*' $O/bench_$i.log)"
  i=$((i+1))
done
if [ "${TRACE:-0}" = 1 ]; then
  env ${V[0]} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
  ms=$(grep -o '"ms_per_step": [0-9.]*' $O/kt.log | grep -o '[0-9.]*$')
  python3 scripts/timeline.py $O $ms > $O/timeline.txt && head -40 $O/timeline.txt
fi
