set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/bp1; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_blat.py tests/test_gpu_s5s6.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $O/bench.log; grep -o '"genome_bwa_s4_s5": [0-9.]*' $O/bench.log
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_blat<" --output-format csv -d $O/fetch -o run -- python3 -u bench.py --steps 1 --warmup 0 --no-cpu > $O/fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_blat<" --output-format csv -d $O/write -o run -- python3 -u bench.py --steps 1 --warmup 0 --no-cpu > $O/write.log 2>&1
python3 - <<'PY'
import csv, glob
for sub in ("fetch", "write"):
    for f in glob.glob(f"gpurun_out/bp1/{sub}/**/*counter_collection.csv", recursive=True):
        tot = {}
        for r in csv.DictReader(open(f)):
            tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0) + float(r["Counter_Value"])
        print(sub, tot)
PY
