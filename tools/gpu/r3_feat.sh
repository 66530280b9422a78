# round-3 feature checks: fused MIL-NCE (split-bf16), fused-distance soft-DTW, full-depth numerics
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-feat}
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_halo.py tests/test_gpu_ops.py -v -s -k "milnce or softdtw or hard_dtw" --timeout 200 --timeout-method thread > $D/pytest.log 2>&1 || true
grep -E "PASS|FAIL|fused:|B [0-9]+:|Error" $D/pytest.log | head -60
timeout -k 10 400 python -u -m pytest tests/test_gpu_fulldepth.py -s -q --timeout 240 --timeout-method thread > $D/fd.log 2>&1 || true
grep -E "out |vs fp32|worst|passed|failed|Error" $D/fd.log | head -40
