set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof19 -o run --output-format csv -- python bench.py --steps 3 --warmup 2 > gpurun_out/prof19.log 2>&1 || { tail -20 gpurun_out/prof19.log; exit 1; }
f=$(find gpurun_out/prof19 -name "run_kernel_trace.csv" | head -1)
python tools/kstats.py $f --skip 2 --top 70 > gpurun_out/prof19_summary.txt
rm -f $f
tail -3 gpurun_out/prof19.log
