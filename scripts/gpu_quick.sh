# quick GPU check: align parity tests + bench (K2 variant chosen by env)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-q}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_align.py -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -15 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --no-cpu --steps 20 > $O/bench.log 2>&1 && tail -1 $O/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'ms', d['ms_per_step'], d['kernels_ms'])" && \
AF_K2_GRP=0 timeout -k 10 200 python bench.py --no-cpu --steps 20 > $O/bench0.log 2>&1 && tail -1 $O/bench0.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('GRP=0 value', d['value'], 'ms', d['ms_per_step'], d['kernels_ms'])"
