# Stem wgrad variants (MILNCE_STEM_WGRAD_V): GPU stem tests under each, then same-box A/B bench
# and a kernel trace of each: bash tools/gpu/stem_wgrad_ab.sh A B
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/stem_wgrad_ab
mkdir -p $D
for v in "$@"; do
  MILNCE_STEM_WGRAD_V=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -m gpu -k "stem" --timeout 120 --timeout-method thread > $D/pytest_v$v.log 2>&1 || { tail -40 $D/pytest_v$v.log; exit 1; }
  tail -1 $D/pytest_v$v.log
done
for r in 1 2; do
  for v in "$@"; do
    echo "== MILNCE_STEM_WGRAD_V=$v round $r"
    MILNCE_STEM_WGRAD_V=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 | cut -c1-160
  done
done > $D/bench.txt 2>&1
grep -v amdgpu.ids $D/bench.txt
for v in "$@"; do
  MILNCE_STEM_WGRAD_V=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof_v$v -o run --output-format csv -- python bench.py --steps 3 --warmup 2 > $D/rocprof_v$v.log 2>&1
  T=$(find $D/prof_v$v -name "run_kernel_trace.csv" | head -1)
  python tools/kstats.py $T --skip 3 --top 80 > $D/kstats_v$v.txt
  grep -E "GPU kernel|stem" $D/kstats_v$v.txt
done
find $D -name "*.csv" -size +20M -delete
