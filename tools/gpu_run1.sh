set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_gpu_ops.py -x -q -m gpu > gpurun_out/pytest_gpu_ops.log 2>&1 || { tail -60 gpurun_out/pytest_gpu_ops.log; exit 1; }
tail -5 gpurun_out/pytest_gpu_ops.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
