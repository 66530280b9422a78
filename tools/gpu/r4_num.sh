# Per-block numerics vs fp32 at random init and on trained weights, pre-BN shift on / off
# (tools/fulldepth_numerics.py -> profiles/r4_fulldepth.md), then the full-depth GPU tests.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-r4num}
mkdir -p $D
timeout -k 10 900 python -u tools/fulldepth_numerics.py --steps ${2:-400} --out $D/r4_fulldepth.md > $D/num.log 2>&1 || { tail -40 $D/num.log; exit 1; }
grep -v amdgpu.ids $D/num.log | tail -40
timeout -k 10 600 python -u -m pytest tests/test_gpu_fulldepth.py -x -v -s -m gpu --timeout 500 --timeout-method thread > $D/fulldepth.log 2>&1 || { tail -40 $D/fulldepth.log; exit 1; }
grep -E "hip:|vs fp32|worst|passed|failed" $D/fulldepth.log
