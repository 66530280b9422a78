# the pool / stem GPU tests only
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pooltests
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q -m gpu -k "pool or stem or gate" --timeout 240 --timeout-method thread > gpurun_out/pooltests/pytest.log 2>&1
rc=$?
tail -3 gpurun_out/pooltests/pytest.log
exit $rc
