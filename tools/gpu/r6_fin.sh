set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6fin
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_ops.py -k "bitwise or bn or finalize or gradcache" > gpurun_out/r6fin/pytest.log 2>&1 || { tail -30 gpurun_out/r6fin/pytest.log; exit 1; }
tail -1 gpurun_out/r6fin/pytest.log
bash tools/gpu/r6_ab.sh r6fin - "MILNCE_LIB_PATH=$GRAFT_REPO_ROOT/mil_nce_howto100m_amd/_native/libmilnce_hip_def_MILNCE_FIN_RG=128.so"
