# Same-box A/B of two library builds (bench A B A B + one kernel trace each):
#   bash tools/gpu/ab_libs.sh TAG LIB_A LIB_B [pytest -k expr run first on the default library]
# LIB_* are file names in mil_nce_howto100m_amd/_native ("default" = libmilnce_hip.so).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; A=$2; B=$3; K=${4:-}
D=gpurun_out/$TAG
N=$GRAFT_REPO_ROOT/mil_nce_howto100m_amd/_native
mkdir -p $D
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu -k "$K" --timeout 240 --timeout-method thread > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
  tail -1 $D/pytest.log
fi
libpath() { if [ "$1" = default ]; then echo ""; else echo "$N/$1"; fi; }
for r in 1 2; do
  for v in "$A" "$B"; do
    echo "== $v round $r"
    MILNCE_LIB_PATH=$(libpath $v) timeout -k 10 300 python bench.py --steps 20 --warmup 5 | cut -c1-160
  done
done > $D/bench.txt 2>&1
grep -v amdgpu.ids $D/bench.txt
for arm in a b; do
  if [ $arm = a ]; then v=$A; else v=$B; fi
  export MILNCE_LIB_PATH=$(libpath $v)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof_$arm -o run --output-format csv -- python bench.py --steps 3 --warmup 2 > $D/prof_$arm.log 2>&1 || { tail -20 $D/prof_$arm.log; exit 1; }
  T=$(find $D/prof_$arm -name "run_kernel_trace.csv" | head -1)
  python tools/kstats.py $T --skip 3 --top 90 > $D/kstats_$arm.txt
  head -3 $D/kstats_$arm.txt
done
find $D -name "*.csv" -size +20M -delete
