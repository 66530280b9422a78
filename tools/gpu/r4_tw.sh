# temporal box wgrad: tests, isolated timings against im2col / halo, counters of the register variant
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-r4tw}
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -m gpu -k "temporal_box_wgrad" --timeout 120 --timeout-method thread > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
timeout -k 10 300 python tools/halo_bench.py > $D/halo_bench.txt 2>&1 || { tail -20 $D/halo_bench.txt; exit 1; }
grep -v amdgpu.ids $D/halo_bench.txt
