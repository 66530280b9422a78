set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof22 -o run --output-format csv -- python tools/pool_bench.py > gpurun_out/prof22.log 2>&1 || { tail -20 gpurun_out/prof22.log; exit 1; }
f=$(find gpurun_out/prof22 -name "run_kernel_stats.csv" | head -1)
cut -d, -f1-8 $f | head -30
