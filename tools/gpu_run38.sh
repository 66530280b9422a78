set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q -m gpu -k "pool or gate or model or direct or bench or stem" --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 600 python bench.py > gpurun_out/bench38.json 2> gpurun_out/bench38.err || { tail -30 gpurun_out/bench38.err; exit 1; }
cat gpurun_out/bench38.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof38 -o run --output-format csv -- python bench.py --steps 3 --warmup 2 > gpurun_out/prof38.log 2>&1 || { tail -20 gpurun_out/prof38.log; exit 1; }
f=$(find gpurun_out/prof38 -name "run_kernel_trace.csv" | head -1)
python tools/kstats.py $f --skip 2 --top 100 > gpurun_out/prof38_summary.txt
rm -f $f
head -3 gpurun_out/prof38_summary.txt
grep -E "maxpool_bwd|bn_bwd_apply" gpurun_out/prof38_summary.txt || true
