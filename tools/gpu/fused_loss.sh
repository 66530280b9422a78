set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/fused
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_halo.py -k milnce -v -s --timeout 200 --timeout-method thread > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
grep -E "fused:|PASS|FAIL|passed|failed" $D/pytest.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k milnce -q --timeout 200 --timeout-method thread > $D/pytest2.log 2>&1 || { tail -40 $D/pytest2.log; exit 1; }
tail -1 $D/pytest2.log
