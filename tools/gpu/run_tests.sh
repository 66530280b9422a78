# Usage: bash tools/gpu/run_tests.sh TAG [pytest -k expr] -- GPU tests in ONE process, then smoke().
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-t}; K=${2:-}
D=gpurun_out/$TAG
mkdir -p $D
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu "${KA[@]}" --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || { tail -60 $D/pytest.log; exit 1; }
tail -3 $D/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -30 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
