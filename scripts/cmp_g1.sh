set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/cmp
timeout -k 10 300 env AF_GPU_LIB=libafgpu_gprof_old.so GPROF_SAVE=gpurun_out/cmp/old.npy PAIRS=4000000 python3 -u scripts/g_prof.py > gpurun_out/cmp/old.log 2>&1 && \
timeout -k 10 300 env AF_GPU_LIB=libafgpu_gprof.so GPROF_SAVE=gpurun_out/cmp/new.npy PAIRS=4000000 python3 -u scripts/g_prof.py > gpurun_out/cmp/new.log 2>&1
rc=$?; grep -h "G1 cycles" gpurun_out/cmp/*.log; exit $rc
