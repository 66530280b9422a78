set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 600 python bench.py > gpurun_out/bench33.json 2> gpurun_out/bench33.err || { tail -30 gpurun_out/bench33.err; exit 1; }
cat gpurun_out/bench33.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof33 -o run --output-format csv -- python bench.py --steps 3 --warmup 2 > gpurun_out/prof33.log 2>&1 || { tail -20 gpurun_out/prof33.log; exit 1; }
f=$(find gpurun_out/prof33 -name "run_kernel_trace.csv" | head -1)
python tools/kstats.py $f --skip 2 --top 80 > gpurun_out/prof33_summary.txt
rm -f $f
head -3 gpurun_out/prof33_summary.txt
grep -E "finalize|maxpool_bwd|gate_bwd" gpurun_out/prof33_summary.txt
