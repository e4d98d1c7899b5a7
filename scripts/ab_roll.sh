set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r02_roll; mkdir -p $O
AF_S2_ROLL=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_c3.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/c3_tests_roll.log 2>&1 || { echo TESTFAIL; tail -30 $O/c3_tests_roll.log; exit 1; }
tail -2 $O/c3_tests_roll.log
run() { tag=$1; shift; timeout -k 10 300 python -u bench.py --no-cpu --steps 8 "$@" > $O/bench_$tag.log 2>&1 || { echo "BENCHFAIL $tag"; tail -20 $O/bench_$tag.log; exit 1; }
  grep '^{' $O/bench_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['ms_per_step'], d['phases_ms']['s2'], d['roofline']['frac'])"; }
run base
AF_S2_ROLL=1 run roll
AF_S2_ROLL=1 run roll_b120 --batch-chunks 120
AF_S2_ROLL=1 run roll_b120_i6 --batch-chunks 120 --inflight 6
AF_S2_ROLL=1 run roll_b160_i3 --batch-chunks 160 --inflight 3
