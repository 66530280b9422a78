# Box kernel extensions: GPU tests, then same-box A/Bs of the prefire and of the N 96 / 160 and
# T = 2 tiles (bash tools/gpu/boxext.sh TAG)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-boxext}
D=gpurun_out/$TAG
mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_box.py > $D/test.txt 2>&1 || { tail -30 $D/test.txt; exit 1; }
tail -3 $D/test.txt
bash tools/gpu/ab_trace.sh $TAG/prefire MILNCE_BOX_PREFIRE 0 1
bash tools/gpu/ab_trace.sh $TAG/ext MILNCE_BOX_EXT 0 1
