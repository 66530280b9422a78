# v4 conv kernels: numerics tests, per-variant timings of the big layers, then the bench.
#   bash tools/gpu/v4_check.sh TAG
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-v4}
mkdir -p $D
timeout -k 10 500 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_dp.py -x -v -k "v4 or bitwise" --timeout 120 --timeout-method thread > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
timeout -k 10 200 python -u tools/conv_impls.py --cin 64 --cout 192 --k 1 3 3 --impls 4 8 9 12 13 > $D/impls.log 2>&1
timeout -k 10 200 python -u tools/conv_impls.py --cin 192 --cout 192 --k 3 1 1 --impls 4 8 9 12 13 >> $D/impls.log 2>&1
timeout -k 10 200 python -u tools/conv_impls.py --cin 128 --cout 192 --k 1 3 3 --hw 25 --impls 4 8 9 12 13 >> $D/impls.log 2>&1
timeout -k 10 200 python -u tools/conv_impls.py --cin 256 --cout 288 --k 1 1 1 --hw 25 --impls 3 4 8 10 >> $D/impls.log 2>&1
cat $D/impls.log
for v in 8,9,10,11 8,9,10,11,12,13 8,9,10,11 8,9,10,11,12,13; do MILNCE_V4_IMPLS=$v timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $D/bench.log 2>&1 || { tail -30 $D/bench.log; exit 1; }; echo "V4_IMPLS=$v"; tail -1 $D/bench.log | cut -c1-120; done
tail -1 $D/bench.log | cut -c1-300
