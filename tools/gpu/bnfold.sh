# Folded BN-backward element op: whole GPU suite, then a same-box A/B against the previous library
# (mil_nce_howto100m_amd/_native/libmilnce_hip_ab.so) (bash tools/gpu/bnfold.sh TAG)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-bnfold}
D=gpurun_out/$TAG
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || { tail -60 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
N=$GRAFT_REPO_ROOT/mil_nce_howto100m_amd/_native
bash tools/gpu/ab_trace.sh $TAG/ab MILNCE_LIB_PATH $N/libmilnce_hip_ab.so $N/libmilnce_hip.so
