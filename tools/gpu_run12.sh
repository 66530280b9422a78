set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --pmc MfmaUtil FETCH_SIZE --kernel-include-regex "conv_" -d gpurun_out/pmc4 -o run --output-format csv -- python tools/conv_bench.py --batch 128 > gpurun_out/pmc4.log 2>&1 || { tail -20 gpurun_out/pmc4.log; exit 1; }
timeout -k 10 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum --kernel-include-regex "conv_" -d gpurun_out/pmc5 -o run --output-format csv -- python tools/conv_bench.py --batch 128 > gpurun_out/pmc5.log 2>&1 || { tail -20 gpurun_out/pmc5.log; exit 1; }
