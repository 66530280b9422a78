set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -m gpu --timeout 200 --timeout-method thread -k "stem" > gpurun_out/pytest_stem.log 2>&1 || { tail -40 gpurun_out/pytest_stem.log; exit 1; }
tail -1 gpurun_out/pytest_stem.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -x -q -m gpu --timeout 250 --timeout-method thread > gpurun_out/pytest_model.log 2>&1 || { tail -40 gpurun_out/pytest_model.log; exit 1; }
tail -1 gpurun_out/pytest_model.log
timeout -k 10 600 python bench.py > gpurun_out/bench29.json 2> gpurun_out/bench29.err || { tail -30 gpurun_out/bench29.err; exit 1; }
cat gpurun_out/bench29.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof29 -o run --output-format csv -- python tools/stem_probe.py > gpurun_out/prof29.log 2>&1 || { tail -20 gpurun_out/prof29.log; exit 1; }
cut -d, -f1-4 $(find gpurun_out/prof29 -name "run_kernel_stats.csv") | grep stem
