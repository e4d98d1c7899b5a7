# round-4: k_g_pe per-pair phases (rescue ksw_align2 / dedup, pairing, records) on the profiling
# build, S4 and S5 in one genome launch (AF_S4_SPLIT=0) so the rows of one call hold both
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-r04g}; mkdir -p $O
AF_S4_SPLIT=0 timeout -k 10 300 python3 -u scripts/g_prof.py > $O/gprof.log 2>&1 || { tail -30 $O/gprof.log; exit 1; }
grep -E "PE|G2 makespan|G1 makespan" $O/gprof.log | head -40
