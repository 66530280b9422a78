# Round-5 quick check: selected GPU tests (pytest -k expr), then bench + one kernel trace.
# bash tools/gpu/r5_quick.sh TAG "pytest-args"
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-r5q}
mkdir -p $D
if [ -n "$2" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread $2 > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
  tail -2 $D/pytest.log
fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $D/bench.log 2>&1 || { tail -30 $D/bench.log; exit 1; }
tail -1 $D/bench.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 2 > $D/prof.log 2>&1 || { tail -20 $D/prof.log; exit 1; }
T=$(find $D/prof -name "run_kernel_trace.csv" | head -1)
python tools/kstats.py $T --skip 3 --top 80 > $D/kstats.txt
find $D -name "*.csv" -size +20M -delete
head -40 $D/kstats.txt
