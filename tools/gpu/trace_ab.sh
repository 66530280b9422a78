# box phase traces of two trace-enabled libraries (default trace lib vs $1) on the conv_2c fwd shapes
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
N=$GRAFT_REPO_ROOT/mil_nce_howto100m_amd/_native
D=gpurun_out/traceab
mkdir -p $D
for lib in libmilnce_hip_trace.so "$1"; do
  echo "== $lib"
  for args in "--cin 64 --cout 192 --k 1 3 3" "--cin 192 --cout 192 --k 3 1 1"; do
    MILNCE_LIB_PATH=$N/$lib timeout -k 10 120 python tools/box_trace.py $args --impl 15 --dir fwd 2>&1 | grep -v amdgpu.ids
  done
done
