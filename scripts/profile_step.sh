# configs[2] profile set (TAG names the output dir): a rocprofv3 kernel trace of the bench
# step, then counter passes (each in a run of its own) on the genome calls and BLAT:
# SQ occupancy / issue / wait counters, then FETCH_SIZE, then WRITE_SIZE.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-prof}; mkdir -p $O
export TMPDIR=/tmp
K=${KREGEX:-k_g_|k_blat|k_s5_check|k_seed_stream|k_s2_}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 -u bench.py --steps 3 --warmup 1 --no-cpu > $O/kt.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --kernel-include-regex "$K" --output-format csv -d $O/sq -o run -- python3 -u bench.py --steps 1 --warmup 0 --no-cpu > $O/sq.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" --output-format csv -d $O/fetch -o run -- python3 -u bench.py --steps 1 --warmup 0 --no-cpu > $O/fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" --output-format csv -d $O/write -o run -- python3 -u bench.py --steps 1 --warmup 0 --no-cpu > $O/write.log 2>&1
rc=$?
echo rc=$rc
grep '^{' $O/kt.log | cut -c1-300
f=$(find $O/kt -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -d, -f1-8 "$f" | head -30
exit $rc
