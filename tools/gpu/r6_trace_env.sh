# One traced bench run under extra environment variables: kernel trace + per-queue class totals +
# the step's tail timeline. bash tools/gpu/r6_trace_env.sh TAG [VAR=VALUE ...]
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-r6trace}
shift
mkdir -p $D
for e in "$@"; do export "$e"; done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $D/bench.log 2>&1 || { tail -20 $D/bench.log; exit 1; }
tail -1 $D/bench.log | cut -c1-120
timeout -k 10 300 rocprofv3 --kernel-trace -d $D/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 2 > $D/prof.log 2>&1 || { tail -20 $D/prof.log; exit 1; }
T=$(find $D/prof -name "run_kernel_trace.csv" | head -1)
python tools/step_classes.py $T > $D/classes.txt
python tools/kstats.py $T --skip 3 --top 80 > $D/kstats.txt
cat $D/classes.txt
