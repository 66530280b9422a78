set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python tools/diag_loss.py 8 > gpurun_out/diag.log 2>&1
MILNCE_FUSE_STEM_POOL=0 timeout -k 10 300 python tools/diag_loss.py 8 >> gpurun_out/diag.log 2>&1
timeout -k 10 300 python tools/diag_loss.py 256 >> gpurun_out/diag.log 2>&1
MILNCE_FUSE_STEM_POOL=0 timeout -k 10 300 python tools/diag_loss.py 256 >> gpurun_out/diag.log 2>&1
grep -v amdgpu.ids gpurun_out/diag.log
