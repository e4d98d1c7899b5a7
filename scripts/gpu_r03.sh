# Round-3 GPU validation, in order of cost (every step under its own time limit, stop at the first
# failure): the new device code's parity tests (genome engine incl. the crafted rescue case, S5
# check / S6 rows, BLAT incl. cap counters, the dist_discover GPU backend, the product's device
# path), smoke, the rest of the GPU suite (configs[3]/[4] shapes, the full-size C3 test), then the
# configs[2] bench line with its kernel trace and K1 counter passes (scripts/profile_c3.sh) and the
# product path end to end at 5 % genome scale and at configs[2] size.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-r03}; mkdir -p $O
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_genome.py tests/test_gpu_s5s6.py tests/test_gpu_blat.py tests/test_gpu_dist.py \
    > $O/gpu_new.log 2>&1 || { tail -40 $O/gpu_new.log; exit 1; }
tail -1 $O/gpu_new.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 1100 $T tests -m gpu > $O/gpu_tests.log 2>&1 || { grep -E "FAILED|Error" $O/gpu_tests.log | head; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
TAG=${TAG:-r03} bash scripts/profile_c3.sh || exit 1
timeout -k 10 900 python -u scripts/e2e_c3.py --pairs 2000000 --scale 0.05 --out $O/e2e_c3_small.json \
    > $O/e2e_small.log 2>&1 || { tail -30 $O/e2e_small.log; exit 1; }
tail -1 $O/e2e_small.log | cut -c1-300
timeout -k 10 1100 python -u scripts/e2e_c3.py --out $O/e2e_c3.json > $O/e2e.log 2>&1 || { tail -30 $O/e2e.log; exit 1; }
tail -1 $O/e2e.log | cut -c1-300
