# quick GPU check: align parity tests + bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-q}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_align.py -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -15 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --no-cpu --steps 20 > $O/bench.log 2>&1 && tail -1 $O/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'ms', d['ms_per_step'], d['kernels_ms'], d['roofline']['frac'])"
