set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu39.log 2>&1 || { tail -40 gpurun_out/pytest_gpu39.log; exit 1; }
tail -1 gpurun_out/pytest_gpu39.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke39.log 2>&1 || { tail -30 gpurun_out/smoke39.log; exit 1; }
tail -1 gpurun_out/smoke39.log
timeout -k 10 600 python bench.py > gpurun_out/bench39.json 2> gpurun_out/bench39.err || { tail -30 gpurun_out/bench39.err; exit 1; }
cat gpurun_out/bench39.json
