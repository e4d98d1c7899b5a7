# round-4: kernel trace of the configs[2] bench and the last step's timeline (scripts/timeline.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${TAG:-r04h}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 -u bench.py --steps 3 --warmup 1 --no-cpu > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
ms=$(grep -o '"ms_per_step": [0-9.]*' $O/kt.log | grep -o '[0-9.]*$')
echo "ms_per_step $ms"
python3 scripts/timeline.py $O $ms > $O/timeline.txt; cat $O/timeline.txt
