set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/halo
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_halo.py -x -q --timeout 120 --timeout-method thread > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
timeout -k 10 400 python tools/conv_bench.py > $D/conv_bench.txt 2>&1 || { tail -20 $D/conv_bench.txt; exit 1; }
cat $D/conv_bench.txt | head -30
