# Round-6 full check: GPU suite (one process) + smoke, a bench run that records the kernel plan
# (bench.py --save_plan), then the bench again from that plan table (no tuning; same plan_hash),
# and a kernel trace of the step. Copy gpurun_out/TAG/gfx950.json to
# mil_nce_howto100m_amd/ops/plans/gfx950.json afterwards (the table shipped with the tree).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-r6full}
mkdir -p $D
if [ "${2:-tests}" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || { tail -60 $D/pytest.log; exit 1; }
  tail -2 $D/pytest.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -30 $D/smoke.log; exit 1; }
  tail -1 $D/smoke.log
fi
MILNCE_PLAN_TABLE=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --save_plan $D/gfx950.json > $D/bench_tuned.log 2>&1 || { tail -30 $D/bench_tuned.log; exit 1; }
tail -1 $D/bench_tuned.log | cut -c1-250
mkdir -p mil_nce_howto100m_amd/ops/plans
cp $D/gfx950.json mil_nce_howto100m_amd/ops/plans/gfx950.json
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $D/bench.log 2>&1 || { tail -30 $D/bench.log; exit 1; }
tail -1 $D/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 2 > $D/prof.log 2>&1 || { tail -20 $D/prof.log; exit 1; }
T=$(find $D/prof -name "run_kernel_trace.csv" | head -1)
python tools/kstats.py $T --skip 3 --top 80 > $D/kstats.txt
python tools/timeline.py $T > $D/timeline.txt
find $D -name "*.csv" -size +20M -delete
head -12 $D/kstats.txt
cat $D/timeline.txt
