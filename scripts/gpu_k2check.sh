# K2 change check: align parity tests + C2 bench (gpu_quick.sh), a 2x150 bench line, placement parity
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-k2c} bash scripts/gpu_quick.sh || exit $?
O=gpurun_out/${TAG:-k2c}
timeout -k 10 200 python bench.py --no-cpu --read-len 150 --steps 20 > $O/bench150.log 2>&1 && \
  tail -1 $O/bench150.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('L150', d['ms_per_step'], d['kernels_ms'])" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_place.py -x -q --timeout 240 --timeout-method thread > $O/place.log 2>&1
rc=$?
tail -2 $O/place.log
exit $rc
