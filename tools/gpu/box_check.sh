# Box-tiled conv (csrc/conv_box.hip): numerics tests, then isolated timings next to v4 (the dgrad
# with the producer-BN partials epilogue, as in the step). bash tools/gpu/box_check.sh TAG
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-box}
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_box.py -x -v --timeout 120 --timeout-method thread > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -3 $D/pytest.log
{
timeout -k 10 120 python tools/conv_impls.py --producer 1 --impls 12 13 14 15
timeout -k 10 120 python tools/conv_impls.py --producer 1 --cin 192 --k 3 1 1 --impls 12 13 14 15
timeout -k 10 120 python tools/conv_impls.py --producer 1 --cin 128 --cout 192 --hw 25 --impls 12 13 14 15
timeout -k 10 120 python tools/conv_impls.py --producer 1 --cin 192 --cout 192 --hw 25 --k 3 1 1 --impls 12 13 14 15
} > $D/conv.txt 2>&1
grep -v amdgpu.ids $D/conv.txt
