# round-4 check C: box / shift numerics, box phase traces, then a same-box A/B of two libraries
#   bash tools/gpu/r4_c.sh TAG LIB_B   (LIB_A = the default library)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-r4c}
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_box.py tests/test_gpu_ops.py -x -v -s -m gpu -k "box or temporal_box_wgrad or stem or producer or fused_bn or bn_prologue or shifted or conv_bn_relu or group" --timeout 240 --timeout-method thread > $D/pytest.log 2>&1 || { grep -E "FAILED|Error|error" $D/pytest.log | head; tail -30 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
grep -h "^out \|shifted .* plain" $D/pytest.log | cut -c1-300 || true
bash tools/gpu/box_trace.sh ${1:-r4c}/trace
bash tools/gpu/ab_libs.sh ${1:-r4c}/ab default $2
