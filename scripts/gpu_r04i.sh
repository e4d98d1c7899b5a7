# round-4: the genome tests first (heavy path forced on every read among them), under a tight
# limit, then the whole suite + smoke + bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-r04i}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_genome.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/genome.log 2>&1 || { tail -30 $O/genome.log; exit 1; }
tail -2 $O/genome.log
TAG=${TAG:-r04i} bash scripts/gpu_all_r04.sh
