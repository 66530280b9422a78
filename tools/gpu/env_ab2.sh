# Same-box A/B of an environment switch: bash tools/gpu/env_ab2.sh TAG "VAR=val [VAR2=val]"
set -e
cd $GRAFT_REPO_ROOT
D=gpurun_out/${1:-envab}
mkdir -p $D
for r in 1 2; do
  for v in base new; do
    echo "== $v round $r"
    if [ $v = new ]; then env $2 timeout -k 10 300 python bench.py --steps 20 --warmup 5 | cut -c1-170
    else timeout -k 10 300 python bench.py --steps 20 --warmup 5 | cut -c1-170; fi
  done
done > $D/bench.txt 2>&1
grep -v amdgpu.ids $D/bench.txt
