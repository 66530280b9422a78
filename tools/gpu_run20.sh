set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -v -m gpu --timeout 300 --timeout-method thread -k "maxpool or inception_head or gate" > gpurun_out/pytest_pool.log 2>&1 || { tail -40 gpurun_out/pytest_pool.log; exit 1; }
tail -2 gpurun_out/pytest_pool.log
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 600 python bench.py > gpurun_out/bench20.json 2> gpurun_out/bench20.err || { tail -30 gpurun_out/bench20.err; exit 1; }
cat gpurun_out/bench20.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof20 -o run --output-format csv -- python bench.py --steps 3 --warmup 2 > gpurun_out/prof20.log 2>&1 || { tail -20 gpurun_out/prof20.log; exit 1; }
f=$(find gpurun_out/prof20 -name "run_kernel_trace.csv" | head -1)
python tools/kstats.py $f --skip 2 --top 70 > gpurun_out/prof20_summary.txt
rm -f $f
head -30 gpurun_out/prof20_summary.txt
