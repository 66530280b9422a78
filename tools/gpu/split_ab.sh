# wave-role split (BOX_SPLIT) A/B: box tests, phase traces (split / no split / stores ablated), bench A/B
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
N=$GRAFT_REPO_ROOT/mil_nce_howto100m_amd/_native
D=gpurun_out/splitab
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_box.py -x -q -m gpu --timeout 240 --timeout-method thread > $D/pytest.log 2>&1 || { grep -E "FAILED|Error" $D/pytest.log | head; tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
for lib in libmilnce_hip_trace.so "libmilnce_hip_def_BOX_TRACE=1,BOX_SPLIT=0.so" "libmilnce_hip_def_BOX_TRACE=1,BOX_ABLATE=16.so"; do
  echo "== $lib"
  for args in "--cin 64 --cout 192 --k 1 3 3" "--cin 192 --cout 192 --k 3 1 1"; do
    MILNCE_LIB_PATH=$N/$lib timeout -k 10 120 python tools/box_trace.py $args --impl 15 --dir fwd 2>&1 | grep -v amdgpu.ids
  done
done > $D/trace.txt
grep -E "==|fwd|wait|barrier|mfma|stage|stores|total" $D/trace.txt
bash tools/gpu/ab_libs.sh splitab/ab default "libmilnce_hip_def_BOX_SPLIT=0.so"
