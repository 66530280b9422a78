# Same-box A/B of alternative library builds (csrc/build.py --define ...) on the flagship bench,
# all arms on the plan table copy given as $2 (the sources' digest differs from the shipped one
# while an A/B macro is in them):  bash tools/gpu/lib_ab.sh TAG PLAN.json LIB_A LIB_B ...
# ("-" = the release library)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-libab}
export MILNCE_PLAN_TABLE=$GRAFT_REPO_ROOT/$2
shift 2
mkdir -p $D
for r in 1 2; do
  for l in "$@"; do
    if [ "$l" = "-" ]; then unset MILNCE_LIB_PATH; else export MILNCE_LIB_PATH=$GRAFT_REPO_ROOT/mil_nce_howto100m_amd/_native/$l; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $D/b.json 2> $D/b.err
    echo "[$l] round $r: $(python -c "import json;d=json.load(open('$D/b.json'));print(d['value'], d['ms_per_step'], d['plan']['source'])")"
  done
done
