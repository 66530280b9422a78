# Same-box A/B of an environment knob over bench.py: bash tools/gpu/env_ab.sh TAG VAR "v1 v2 ..." [pytest -k]
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; VAR=$2; VALS=$3; K=${4:-}
D=gpurun_out/$TAG
mkdir -p $D
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu -k "$K" --timeout 240 --timeout-method thread > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
  tail -1 $D/pytest.log
fi
for r in 1 2; do
  for v in $VALS; do
    echo "== $VAR=$v round $r: $(env $VAR=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>&1 | grep metric | cut -c60-150)"
  done
done | tee $D/bench.txt
