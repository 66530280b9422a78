# Same-box A/B of the in-tree library against mil_nce_howto100m_amd/_native/libmilnce_hip_base.so
# (the previous commit's build, made on the host: git stash; python csrc/build.py; cp ...; git stash pop;
# python csrc/build.py): GPU tests of the new build first. bash tools/gpu/ab_lib.sh TAG "pytest -k expr"
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-ab_lib}
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu -k "$2" --timeout 200 --timeout-method thread > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
for r in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export MILNCE_LIB_PATH=$GRAFT_REPO_ROOT/mil_nce_howto100m_amd/_native/libmilnce_hip_base.so; else unset MILNCE_LIB_PATH; fi
    echo "== $v round $r"
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 | cut -c1-160
  done
done > $D/bench.txt 2>&1
grep -v amdgpu.ids $D/bench.txt
