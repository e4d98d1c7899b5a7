# A round's profile set at the current commit (TAG names gpurun_out/<TAG>): profile_step.sh's
# kernel trace and SQ / FETCH_SIZE / WRITE_SIZE passes, the step timeline, the per-read genome
# profile (libafgpu_gprof.so) and BLAT's per-query phases (libafgpu_prof.so); then, on the host,
# scripts/summarize_prof.py gpurun_out/<TAG> profiles/rNN gpurun_out/<TAG>/bench_line.json.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${TAG:-prof}; O=gpurun_out/$T
TAG=$T bash scripts/profile_step.sh > $O.txt 2>&1 || { tail -20 $O.txt; exit 1; }
grep '^{' $O/kt.log | head -1 > $O/bench_line.json
ms=$(grep -o '"ms_per_step": [0-9.]*' $O/kt.log | grep -o '[0-9.]*$')
python3 scripts/timeline.py $O $ms > $O/timeline.txt
timeout -k 10 400 python3 -u scripts/g_prof.py > $O/gprof.txt 2>&1 || { tail -20 $O/gprof.txt; exit 1; }
timeout -k 10 400 python3 -u scripts/blat_prof.py 50000000 $O/blat_phases.json > $O/blat_prof.log 2>&1 || { tail -20 $O/blat_prof.log; exit 1; }
cut -c1-200 $O/bench_line.json
