set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q -m gpu --timeout 300 --timeout-method thread -k "maxpool or inception_head or gate" > gpurun_out/pytest_pool.log 2>&1 || { tail -40 gpurun_out/pytest_pool.log; exit 1; }
tail -1 gpurun_out/pytest_pool.log
timeout -k 10 600 python tools/pool_bench.py > gpurun_out/pool_bench.txt 2>&1 || { tail -30 gpurun_out/pool_bench.txt; exit 1; }
cat gpurun_out/pool_bench.txt
