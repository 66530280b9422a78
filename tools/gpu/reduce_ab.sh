# wgrad slab reduction rewrite: conv / stem / halo GPU tests, then same-box A/B bench against the
# previous commit's library (built here from git into libmilnce_hip_ab.so): bash tools/gpu/reduce_ab.sh
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/reduce_ab
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_halo.py -x -q -m gpu -k "conv or stem or halo or wgrad" --timeout 200 --timeout-method thread > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
for r in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export MILNCE_LIB_PATH=$GRAFT_REPO_ROOT/mil_nce_howto100m_amd/_native/libmilnce_hip_base.so; else unset MILNCE_LIB_PATH; fi
    echo "== $v round $r"
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 | cut -c1-160
  done
done > $D/bench.txt 2>&1
grep -v amdgpu.ids $D/bench.txt
