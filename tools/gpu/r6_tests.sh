# GPU test suite without -x (every failure listed), one process; then smoke.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-r6tests}
mkdir -p $D
timeout -k 10 1000 python -u -m pytest tests/ -q -m gpu --timeout 300 --timeout-method thread ${2:-} > $D/pytest.log 2>&1 || { grep -E "^(FAILED|ERROR)|passed|failed" $D/pytest.log | tail -40; exit 1; }
tail -2 $D/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -30 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
