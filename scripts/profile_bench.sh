set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/${PROF_TAG:-prof}
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${PROF_TAG:-prof}/kt -o run -- python3 bench.py --steps 40 --warmup 5 --no-cpu > gpurun_out/${PROF_TAG:-prof}/bench.log 2>&1 && \
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${PROF_TAG:-prof}/pmc_fetch -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/${PROF_TAG:-prof}/pmc1.log 2>&1 && \
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${PROF_TAG:-prof}/pmc_write -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/${PROF_TAG:-prof}/pmc2.log 2>&1 && \
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${PROF_TAG:-prof}/pmc_sq -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/${PROF_TAG:-prof}/pmc3.log 2>&1
echo "rc=$?"
find gpurun_out/${PROF_TAG:-prof} -name "*.csv" | head -20
