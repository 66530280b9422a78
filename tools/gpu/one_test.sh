# one pytest -k expression on the GPU (verbose, prints)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/onetest
timeout -k 10 600 python -u -m pytest tests/ -x -v -s -m gpu -k "$1" --timeout 300 --timeout-method thread > gpurun_out/onetest/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|SKIPPED|Error|assert" gpurun_out/onetest/pytest.log | head -30
tail -2 gpurun_out/onetest/pytest.log
exit $rc
