# Same-box A/B of a runtime switch: bash tools/gpu/ab_env.sh TAG VAR VALUE_A VALUE_B [pytest -k expr]
# Optional GPU tests first, then interleaved bench runs A B A B (box-to-box variance is larger
# than most of the effects measured this way).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; VAR=$2; A=$3; B=$4; K=${5:-}
D=gpurun_out/$TAG
mkdir -p $D
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu -k "$K" --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || { tail -60 $D/pytest.log; exit 1; }
  tail -3 $D/pytest.log
fi
for r in 1 2; do
  for v in "$A" "$B"; do
    echo "== $VAR=$v round $r"
    env $VAR=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 | cut -c1-160
  done
done > $D/bench.txt 2>&1
cat $D/bench.txt
