set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/halo
mkdir -p $D
timeout -k 10 300 python -m pytest tests/test_gpu_halo.py -x -q > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
timeout -k 10 300 python tools/halo_bench.py > $D/halo_bench.txt 2>&1 || { tail -20 $D/halo_bench.txt; exit 1; }
cat $D/halo_bench.txt
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU -d $D/pa -o run --output-format csv -- python tools/halo_bench.py > $D/pa.log 2>&1 || { tail -5 $D/pa.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE SQ_INSTS_VMEM -d $D/pb -o run --output-format csv -- python tools/halo_bench.py > $D/pb.log 2>&1 || { tail -5 $D/pb.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace -d $D/pt -o run --output-format csv -- python tools/halo_bench.py > $D/pt.log 2>&1 || { tail -5 $D/pt.log; exit 1; }
python tools/pmc_kernels.py $D > $D/pmc.txt
grep -A 30 "halo_wgrad" $D/pmc.txt | grep -E "==|wait|clock|mfma|conflict|INSTS_(VALU|MFMA|LDS)" | head -60
