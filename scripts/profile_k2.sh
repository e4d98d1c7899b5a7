# rocprofv3 counter passes on the bench step (K2 rows are the k_align dispatches)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${PROF_TAG:-k2prof}; mkdir -p $O
export TMPDIR=/tmp
P="timeout -k 10 300 rocprofv3 --output-format csv"
$P --kernel-trace --stats -d $O/kt -o run -- python3 scripts/k2_probe.py > $O/kt.log 2>&1 && \
$P --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD -d $O/p1 -o run -- python3 scripts/k2_probe.py > $O/p1.log 2>&1 && \
$P --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA -d $O/p2 -o run -- python3 scripts/k2_probe.py > $O/p2.log 2>&1 && \
$P --pmc SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $O/p3 -o run -- python3 scripts/k2_probe.py > $O/p3.log 2>&1
echo "rc=$?"
