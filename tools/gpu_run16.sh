set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_ops.py -q -x -k "variants_bitwise" > gpurun_out/pytest_bitwise.log 2>&1 || { tail -30 gpurun_out/pytest_bitwise.log; exit 1; }
tail -2 gpurun_out/pytest_bitwise.log
bash tools/gpu_run15.sh
