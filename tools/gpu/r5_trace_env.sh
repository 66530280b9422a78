# kernel trace of bench.py under an environment: bash tools/gpu/r5_trace_env.sh TAG "VAR=val ..."
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-r5tr}
mkdir -p $D
export $2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 2 > $D/prof.log 2>&1 || { tail -20 $D/prof.log; exit 1; }
T=$(find $D/prof -name "run_kernel_trace.csv" | head -1)
python tools/kstats.py $T --skip 3 --top 80 > $D/kstats.txt
find $D -name "*.csv" -size +40M -delete
head -8 $D/kstats.txt
