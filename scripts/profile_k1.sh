# rocprofv3 counter passes on K1 only (each --pmc group is its own pass)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${PROF_TAG:-k1prof}; mkdir -p $O
export TMPDIR=/tmp
rocprofv3 -L > $O/counters_list.txt 2>&1 || true
timeout -k 10 300 python3 scripts/k1_probe.py > $O/probe.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 scripts/k1_probe.py > $O/kt.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD --output-format csv -d $O/p1 -o run -- python3 scripts/k1_probe.py > $O/p1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $O/p2 -o run -- python3 scripts/k1_probe.py > $O/p2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_BRANCH GRBM_GUI_ACTIVE --output-format csv -d $O/p3 -o run -- python3 scripts/k1_probe.py > $O/p3.log 2>&1
echo "rc=$?"; cat $O/probe.log
