set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gradcache.py -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu50.log 2>&1 || { tail -40 gpurun_out/pytest_gpu50.log; exit 1; }
tail -3 gpurun_out/pytest_gpu50.log
