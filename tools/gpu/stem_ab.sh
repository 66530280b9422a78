# Stem kernel variants: GPU stem tests under both, then same-box A/B bench (MILNCE_STEM_FWD_V and
# MILNCE_STEM_WGRAD_V 0 / 1)
# and one bench with torch-profiler stacks of the small ATen ops: bash tools/gpu/stem_ab.sh
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/stem_ab
mkdir -p $D
for v in 1 0; do
  MILNCE_STEM_FWD_V=$v MILNCE_STEM_WGRAD_V=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -m gpu -k "stem" --timeout 120 --timeout-method thread > $D/pytest_v$v.log 2>&1 || { tail -40 $D/pytest_v$v.log; exit 1; }
  tail -1 $D/pytest_v$v.log
done
for r in 1 2; do
  for v in 0 1; do
    echo "== MILNCE_STEM_FWD_V=$v round $r"
    MILNCE_STEM_FWD_V=$v MILNCE_STEM_WGRAD_V=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 | cut -c1-160
  done
done > $D/bench.txt 2>&1
cat $D/bench.txt
timeout -k 10 300 python bench.py --steps 3 --warmup 2 --profile_steps 1 > $D/prof_bench.txt 2>&1
cp gpurun_out/torch_profile*.txt $D/ 2>/dev/null || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 2 > $D/rocprof.log 2>&1
T=$(find $D/prof -name "run_kernel_trace.csv" | head -1)
python tools/kstats.py $T --skip 3 --top 80 > $D/kstats.txt
find $D -name "*.csv" -size +20M -delete
grep -E "GPU kernel|stem" $D/kstats.txt
