# Row-sweep stride-1 pool: GPU pool tests, then tools/pool_bench.py over (MILNCE_S1_G, _DF, _DB).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-r6pool}
mkdir -p $D
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "maxpool or inception_head" > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
timeout -k 10 200 python -u tools/pool_bench.py > $D/base.log 2>&1 || { cat $D/base.log; exit 1; }
cat $D/base.log
for cfg in ${2:-"4 1 1" "4 2 2" "4 3 2" "4 4 2" "2 3 2" "8 3 2"}; do
  set -- $cfg
  MILNCE_S1_G=$1 MILNCE_S1_DF=$2 MILNCE_S1_DB=$3 timeout -k 10 200 python -u tools/pool_bench.py --impls 2 > $D/g$1_$2_$3.log 2>&1 || { cat $D/g$1_$2_$3.log; exit 1; }
  echo "G=$1 DF=$2 DB=$3"; grep rows $D/g$1_$2_$3.log
done
