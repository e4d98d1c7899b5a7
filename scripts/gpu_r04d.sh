# round-4: G1 per-phase profile; the full-size configs[2] test (bwa-index checks at 3.09 Gbp, exact
# reads beyond 2^31); the configs[3] rank test through dist_discover over a one-rank RCCL group
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-r04d}; mkdir -p $O
T="python -u -m pytest -x -v -s --timeout 600 --timeout-method thread"
timeout -k 10 300 python3 -u scripts/g_prof.py > $O/gprof.log 2>&1 || { tail -30 $O/gprof.log; exit 1; }
grep -E "G1|fwd|cycles per" $O/gprof.log | head -30
timeout -k 10 700 $T tests/test_gpu_c3.py -k full_size > $O/c3_full.log 2>&1 || { tail -40 $O/c3_full.log; exit 1; }
grep -E "index checks|exact reads|passed|failed" $O/c3_full.log
timeout -k 10 600 $T tests/test_gpu_configs.py -k configs3 > $O/configs3.log 2>&1 || { tail -40 $O/configs3.log; exit 1; }
tail -1 $O/configs3.log
