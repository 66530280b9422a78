# s1 pool LDS layout: isolated bandwidth (tools/ew_bench.py) with the previous and the new library,
# then the step A/B (bash tools/gpu/pool_ab.sh TAG)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-poolab}
D=gpurun_out/$TAG
mkdir -p $D
N=$GRAFT_REPO_ROOT/mil_nce_howto100m_amd/_native
for L in libmilnce_hip_ab.so libmilnce_hip.so; do
  echo "== $L"
  MILNCE_LIB_PATH=$N/$L timeout -k 10 300 python tools/ew_bench.py 2>&1 | grep -i "s1" || true
done > $D/ew.txt 2>&1
cat $D/ew.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "pool" > $D/test.txt 2>&1 || { tail -30 $D/test.txt; exit 1; }
tail -2 $D/test.txt
bash tools/gpu/ab_trace.sh $TAG/ab MILNCE_LIB_PATH $N/libmilnce_hip_ab.so $N/libmilnce_hip.so
