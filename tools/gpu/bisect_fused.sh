# one GPU test under shift on/off and two libraries (default / $2): which change moved it
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/bisect
mkdir -p $D
K=${1:-fused_bn_backward_partials}
N=$GRAFT_REPO_ROOT/mil_nce_howto100m_amd/_native
for lib in default $2; do
  for s in 1 0; do
    if [ $lib = default ]; then export MILNCE_LIB_PATH=""; else export MILNCE_LIB_PATH=$N/$lib; fi
    MILNCE_BN_SHIFT=$s timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_box.py -x -q -m gpu -k "$K" --timeout 240 --timeout-method thread > $D/$lib.$s.log 2>&1
    echo "$lib shift=$s rc=$? $(tail -1 $D/$lib.$s.log)"
  done
done
