# whole GPU suite (one process) + smoke + bench + kernel trace + PMC of the step's top kernels
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-r3full}
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || { tail -60 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -30 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $D/bench.log 2>&1 || { tail -30 $D/bench.log; exit 1; }
tail -1 $D/bench.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 2 > $D/prof.log 2>&1 || { tail -20 $D/prof.log; exit 1; }
T=$(find $D/prof -name "run_kernel_trace.csv" | head -1)
python tools/kstats.py $T --skip 3 --top 80 > $D/kstats.txt
find $D -name "*.csv" -size +20M -delete
head -30 $D/kstats.txt
