set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke48.log 2>&1 || { tail -30 gpurun_out/smoke48.log; exit 1; }
tail -1 gpurun_out/smoke48.log
D=gpurun_out/pmc48
mkdir -p $D
timeout -s KILL 180 rocprofv3 --kernel-trace -d $D/t -o run --output-format csv -- python bench.py --steps 1 --warmup 1 > $D/t.log 2>&1 || { tail -5 $D/t.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc MfmaUtil -d $D/a -o run --output-format csv -- python bench.py --steps 1 --warmup 1 > $D/a.log 2>&1 || { tail -5 $D/a.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $D/b -o run --output-format csv -- python bench.py --steps 1 --warmup 1 > $D/b.log 2>&1 || { tail -5 $D/b.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $D/c -o run --output-format csv -- python bench.py --steps 1 --warmup 1 > $D/c.log 2>&1 || { tail -5 $D/c.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $D/d -o run --output-format csv -- python bench.py --steps 1 --warmup 1 > $D/d.log 2>&1 || { tail -5 $D/d.log; exit 1; }
T=$(find $D/t -name "run_kernel_trace.csv" | head -1)
P=$(find $D/a $D/b $D/c $D/d -name "run_counter_collection.csv")
python tools/pmc_step.py --trace $T --pmc $P --top 60 > $D/summary.txt
find $D -name "*.csv" -size +20M -delete
cat $D/summary.txt | head -30
