# Branch streams (MILNCE_BRANCH_STREAMS=1): model-level GPU tests under it, then a same-plan A/B.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-r6branch}
mkdir -p $D
MILNCE_BRANCH_STREAMS=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_training.py > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
bash tools/gpu/r6_ab.sh $1_ab - MILNCE_BRANCH_STREAMS=1
