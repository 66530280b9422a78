set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -m gpu --timeout 200 --timeout-method thread -k "conv" > gpurun_out/pytest_c.log 2>&1 || { tail -40 gpurun_out/pytest_c.log; exit 1; }
tail -1 gpurun_out/pytest_c.log
timeout -k 10 600 python tools/conv_bench.py > gpurun_out/conv_bench28.txt 2>&1 || { tail -20 gpurun_out/conv_bench28.txt; exit 1; }
head -12 gpurun_out/conv_bench28.txt; tail -1 gpurun_out/conv_bench28.txt
