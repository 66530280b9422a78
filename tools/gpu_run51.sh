# Final round-1 check: whole GPU suite in one process, then smoke().
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu51.log 2>&1 || { tail -40 gpurun_out/pytest_gpu51.log; exit 1; }
tail -1 gpurun_out/pytest_gpu51.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke51.log 2>&1 || { tail -30 gpurun_out/smoke51.log; exit 1; }
tail -1 gpurun_out/smoke51.log
