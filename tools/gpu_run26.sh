set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -m gpu --timeout 200 --timeout-method thread -k "stem" > gpurun_out/pytest_stem.log 2>&1 || { tail -40 gpurun_out/pytest_stem.log; exit 1; }
tail -1 gpurun_out/pytest_stem.log
timeout -k 10 600 python bench.py > gpurun_out/bench26.json 2> gpurun_out/bench26.err || { tail -30 gpurun_out/bench26.err; exit 1; }
cat gpurun_out/bench26.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof26 -o run --output-format csv -- python bench.py --steps 3 --warmup 2 > gpurun_out/prof26.log 2>&1 || { tail -20 gpurun_out/prof26.log; exit 1; }
f=$(find gpurun_out/prof26 -name "run_kernel_trace.csv" | head -1)
python tools/kstats.py $f --skip 2 --top 70 > gpurun_out/prof26_summary.txt
rm -f $f
grep -i "stem\|wgrad" gpurun_out/prof26_summary.txt | head
head -3 gpurun_out/prof26_summary.txt
