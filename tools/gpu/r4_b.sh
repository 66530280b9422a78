# round-4 check B: box / twgrad numerics, box phase traces, halo/twgrad timings, bench + kernel trace
#   bash tools/gpu/r4_b.sh TAG ["extra pytest -k expression for tests/test_gpu_ops.py"]
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-r4b}
K=${2:-"temporal_box_wgrad or stem or producer or fused_bn or bn_prologue or shifted or conv_bn_relu or group"}
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_box.py tests/test_gpu_ops.py -x -v -m gpu -k "box or $K" --timeout 240 --timeout-method thread > $D/pytest.log 2>&1 || { tail -60 $D/pytest.log; exit 1; }
tail -3 $D/pytest.log
bash tools/gpu/box_trace.sh ${1:-r4b}/trace
timeout -k 10 300 python tools/halo_bench.py > $D/halo_bench.txt 2>&1 || { tail -20 $D/halo_bench.txt; exit 1; }
grep -v amdgpu.ids $D/halo_bench.txt
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $D/bench.log 2>&1 || { tail -30 $D/bench.log; exit 1; }
tail -1 $D/bench.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 2 > $D/prof.log 2>&1 || { tail -20 $D/prof.log; exit 1; }
T=$(find $D/prof -name "run_kernel_trace.csv" | head -1)
python tools/kstats.py $T --skip 3 --top 90 > $D/kstats.txt
find $D -name "*.csv" -size +20M -delete
head -40 $D/kstats.txt
