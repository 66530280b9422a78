# pre-BN shift A/B on the fusion-equality and shift tests (prints the measured differences)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/shiftdbg
for s in 0 1; do
MILNCE_BN_SHIFT=$s timeout -k 10 300 python -u -m pytest tests/test_gpu_box.py -x -v -s -m gpu -k "inception_head_prologue or prologue_fusion_bitwise" --timeout 240 --timeout-method thread > gpurun_out/shiftdbg/box$s.log 2>&1; echo "shift $s rc=$?"
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -v -s -m gpu -k "shifted" --timeout 240 --timeout-method thread > gpurun_out/shiftdbg/on.log 2>&1; echo "on rc=$?"
grep -hE "passed|failed|^out |shifted .* plain" gpurun_out/shiftdbg/*.log
