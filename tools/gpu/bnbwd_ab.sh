# box tests, then same-box A/B of the BN-backward dgrad prologue (MILNCE_BNBWD_FUSE) with traces
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-bnbwd}
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_box.py -x -v --timeout 120 --timeout-method thread > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -3 $D/pytest.log
bash tools/gpu/ab_trace.sh ${1:-bnbwd} MILNCE_BNBWD_FUSE 0 1
