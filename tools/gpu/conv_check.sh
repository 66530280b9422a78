# conv kernel tests + flagship bench: bash tools/gpu/conv_check.sh TAG
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-cc}
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q -k "conv or stem or inception" --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $D/bench.log 2>&1 || { tail -30 $D/bench.log; exit 1; }
tail -1 $D/bench.log | cut -c1-220
