# Full GPU suite + bench + kernel trace with side-input prefetch in every quad pool backward mode.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu47.log 2>&1 || { tail -40 gpurun_out/pytest_gpu47.log; exit 1; }
tail -1 gpurun_out/pytest_gpu47.log
timeout -k 10 600 python bench.py > gpurun_out/bench47.json 2> gpurun_out/bench47.err || { tail -30 gpurun_out/bench47.err; exit 1; }
cat gpurun_out/bench47.json
D=gpurun_out/prof47
timeout -k 10 300 rocprofv3 --kernel-trace -d $D -o run --output-format csv -- python bench.py --steps 3 --warmup 2 > $D.log 2>&1 || { tail -20 $D.log; exit 1; }
f=$(find $D -name "run_kernel_trace.csv" | head -1)
python tools/kstats.py $f --skip 2 --top 100 > ${D}_summary.txt
rm -f $f
grep -E "GPU kernel|maxpool_bwd_t" ${D}_summary.txt
