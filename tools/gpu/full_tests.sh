# the whole GPU test suite (as the driver runs it), log under gpurun_out/TAG
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-fulltests}
mkdir -p $D
timeout -k 10 1100 python -u -m pytest tests/ -v -m gpu --timeout 300 --timeout-method thread ${2:-} > $D/pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $D/pytest.log | head -30
tail -3 $D/pytest.log
exit $rc
