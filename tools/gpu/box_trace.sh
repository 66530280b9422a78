# Phase timestamps of the box-tiled conv kernels (tools/box_trace.py) on the conv_2c shapes.
# Needs mil_nce_howto100m_amd/_native/libmilnce_hip_trace.so (python csrc/build.py --trace).
#   bash tools/gpu/box_trace.sh TAG
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-boxtrace}
mkdir -p $D
export MILNCE_LIB_PATH=$GRAFT_REPO_ROOT/mil_nce_howto100m_amd/_native/libmilnce_hip_trace.so
{
timeout -k 10 120 python tools/box_trace.py --cin 64 --cout 192 --k 1 3 3 --impl 15 --dir fwd
timeout -k 10 120 python tools/box_trace.py --cin 192 --cout 192 --k 3 1 1 --impl 15 --dir fwd
timeout -k 10 120 python tools/box_trace.py --cin 64 --cout 192 --k 1 3 3 --impl 15 --dir dgrad
timeout -k 10 120 python tools/box_trace.py --cin 192 --cout 192 --k 3 1 1 --impl 15 --dir dgrad
timeout -k 10 120 python tools/box_trace.py --cin 128 --cout 192 --k 1 3 3 --hw 25 --impl 15 --dir fwd
timeout -k 10 120 python tools/box_trace.py --cin 128 --cout 128 --k 1 3 3 --hw 25 --impl 14 --dir fwd
} > $D/trace.txt 2>&1
grep -v amdgpu.ids $D/trace.txt
