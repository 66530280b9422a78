# stem forward variant 2 (all channels per wave): stem tests under it, then timings v1 / v2 / v1 / v2
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/stemv2
mkdir -p $D
MILNCE_STEM_FWD_V=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q -m gpu -k "stem" --timeout 240 --timeout-method thread > $D/pytest.log 2>&1 || { tail -40 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
for r in 1 2; do for v in 1 2; do
  echo "v$v: $(MILNCE_STEM_FWD_V=$v timeout -k 10 120 python tools/stem_fwd_ab.py 2>&1 | grep -v amdgpu)"
done; done
for v in 1 2; do
  echo "bench v$v: $(MILNCE_STEM_FWD_V=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>&1 | grep metric | cut -c60-140)"
done
