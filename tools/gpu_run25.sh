set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q -m gpu --timeout 300 --timeout-method thread -k "wgrad or conv or synth" > gpurun_out/pytest_w.log 2>&1 || { tail -40 gpurun_out/pytest_w.log; exit 1; }
tail -1 gpurun_out/pytest_w.log
timeout -k 10 600 python tools/conv_bench.py > gpurun_out/conv_bench25.txt 2>&1 || { tail -20 gpurun_out/conv_bench25.txt; exit 1; }
timeout -k 10 600 python bench.py > gpurun_out/bench25.json 2> gpurun_out/bench25.err || { tail -30 gpurun_out/bench25.err; exit 1; }
cat gpurun_out/bench25.json
