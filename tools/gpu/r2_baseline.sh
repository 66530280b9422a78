# Round-2 baseline: flagship bench + per-kernel trace of 3 steps.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r2_base
mkdir -p $D
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $D/bench.log 2>&1 || { tail -30 $D/bench.log; exit 1; }
tail -1 $D/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 2 > $D/prof.log 2>&1 || { tail -20 $D/prof.log; exit 1; }
T=$(find $D/prof -name "run_kernel_trace.csv" | head -1)
python tools/kstats.py $T --skip 3 --top 70 > $D/kstats.txt
find $D -name "*.csv" -size +20M -delete
head -40 $D/kstats.txt
