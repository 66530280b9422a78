# halo / conv GPU tests, then bench + kernel trace of the step: bash tools/gpu/halo_step.sh TAG
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-halostep}
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_halo.py tests/test_gpu_ops.py -x -q -m gpu -k "halo or wgrad or stem or conv_bn or shifted or producer or dgrad or fused or v4 or v3" --timeout 240 --timeout-method thread > $D/pytest.log 2>&1 || { tail -60 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $D/bench.log 2>&1 || { tail -30 $D/bench.log; exit 1; }
tail -1 $D/bench.log | cut -c1-300
timeout -k 10 120 python tools/stem_fwd_ab.py >> $D/bench.log 2>&1
tail -1 $D/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 2 > $D/prof.log 2>&1 || { tail -20 $D/prof.log; exit 1; }
T=$(find $D/prof -name "run_kernel_trace.csv" | head -1)
python tools/kstats.py $T --skip 3 --top 90 > $D/kstats.txt
find $D -name "*.csv" -size +20M -delete
head -40 $D/kstats.txt
