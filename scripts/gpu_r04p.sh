# round-4 profile refresh: profile_r04.sh (kernel trace + SQ / FETCH_SIZE passes of the configs[2]
# bench), the last step's timeline, the per-read genome-call profile and the BLAT phase profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-r04p}
TAG=${TAG:-r04p} bash scripts/profile_r04.sh || exit 1
ms=$(grep -o '"ms_per_step": [0-9.]*' $O/kt.log | grep -o '[0-9.]*$')
python3 scripts/timeline.py $O $ms > $O/timeline.txt; grep -v "rocclr\|rocprim\|at::native" $O/timeline.txt
AF_S4_SPLIT=0 timeout -k 10 300 python3 -u scripts/g_prof.py > $O/gprof.log 2>&1 || { tail -30 $O/gprof.log; exit 1; }
timeout -k 10 300 python3 -u scripts/blat_prof.py 50000000 $O/blat_phases_c3.json > $O/blat_prof.log 2>&1 || { tail -30 $O/blat_prof.log; exit 1; }
tail -3 $O/blat_prof.log
WORLD=c3 PAIRS=8000000 READ_LEN=150 timeout -k 10 300 python3 -u scripts/s2_prof.py > $O/s2_prof.log 2>&1 || { tail -30 $O/s2_prof.log; exit 1; }
tail -25 $O/s2_prof.log
