# round-4 refresh: kernel trace + counter passes of the current step, the BLAT per-query phases,
# the genome / BLAT / pipeline GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r04q} bash scripts/profile_r04.sh || exit 1
O=gpurun_out/${TAG:-r04q}
timeout -k 10 300 python3 -u scripts/blat_prof.py 50000000 $O/blat_prof.json > $O/blat_prof.log 2>&1 || { tail -20 $O/blat_prof.log; exit 1; }
head -30 $O/blat_prof.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_pipeline.py tests/test_gpu_dist.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
