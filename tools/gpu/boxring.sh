# Box kernel ring rework: GPU tests, then a same-box A/B against a library built with the previous
# box kernel (mil_nce_howto100m_amd/_native/libmilnce_hip_ab.so) (bash tools/gpu/boxring.sh TAG)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-boxring}
D=gpurun_out/$TAG
mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_box.py > $D/test.txt 2>&1 || { tail -30 $D/test.txt; exit 1; }
tail -3 $D/test.txt
N=$GRAFT_REPO_ROOT/mil_nce_howto100m_amd/_native
bash tools/gpu/ab_trace.sh $TAG/ab MILNCE_LIB_PATH $N/libmilnce_hip_ab.so $N/libmilnce_hip.so
