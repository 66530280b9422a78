cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for r in 1 2; do
  for v in prio noprio; do
    if [ $v = noprio ]; then export MILNCE_LIB_PATH=$GRAFT_REPO_ROOT/mil_nce_howto100m_amd/_native/libmilnce_hip_noprio.so; else unset MILNCE_LIB_PATH; fi
    echo "== $v round $r"
    timeout -k 10 120 python tools/conv_impls.py --impls 4 || exit 1
    timeout -k 10 120 python tools/conv_impls.py --cin 192 --k 3 1 1 --impls 4 || exit 1
  done
done > gpurun_out/ab/conv.txt 2>&1
for v in prio noprio; do
  if [ $v = noprio ]; then export MILNCE_LIB_PATH=$GRAFT_REPO_ROOT/mil_nce_howto100m_amd/_native/libmilnce_hip_noprio.so; else unset MILNCE_LIB_PATH; fi
  echo "== bench $v"
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 | cut -c1-160 || exit 1
done > gpurun_out/ab/bench.txt 2>&1
grep -v amdgpu.ids gpurun_out/ab/conv.txt; cat gpurun_out/ab/bench.txt | grep -v amdgpu.ids
