# Stem wgrad from the pooled gradient (MILNCE_STEM_POOL_WGRAD 1 / 0): stem + conv variant GPU
# tests, same-box A/B bench, kernel trace of the default: bash tools/gpu/stem_pool_ab.sh
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/stem_pool_ab
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -q -m gpu -k "stem or variants or every_tile" --timeout 200 --timeout-method thread > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
for r in 1 2; do
  for v in 0 1; do
    echo "== MILNCE_STEM_POOL_WGRAD=$v round $r"
    MILNCE_STEM_POOL_WGRAD=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 | cut -c1-160
  done
done > $D/bench.txt 2>&1
grep -v amdgpu.ids $D/bench.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 2 > $D/rocprof.log 2>&1
T=$(find $D/prof -name "run_kernel_trace.csv" | head -1)
python tools/kstats.py $T --skip 3 --top 80 > $D/kstats.txt
find $D -name "*.csv" -size +20M -delete
grep -E "GPU kernel|stem|maxpool_bwd_t<1, 3, 3" $D/kstats.txt
