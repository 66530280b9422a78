# Same-box A/B of a compile-time kernel option: bash tools/gpu/ab_define.sh -DV3_PRIO_DEFAULT=0
# Builds conv.hip with the extra define into libmilnce_hip_ab.so (other objects from build/obj or
# a fresh build), then interleaves tools/conv_impls.py runs and one bench per library.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/ab
mkdir -p $D /tmp/abobj
python csrc/build.py > /dev/null
/opt/rocm/bin/hipcc --offload-arch=gfx950 -std=c++17 -fPIC -Icsrc -Wno-unused-result -O3 "$@" -c csrc/conv.hip -o /tmp/abobj/conv.o
AB=$GRAFT_REPO_ROOT/mil_nce_howto100m_amd/_native/libmilnce_hip_ab.so
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $AB $(ls build/obj/*.o | grep -v /conv.o) /tmp/abobj/conv.o
for r in 1 2; do
  for v in base ab; do
    if [ $v = ab ]; then export MILNCE_LIB_PATH=$AB; else unset MILNCE_LIB_PATH; fi
    echo "== $v round $r"
    timeout -k 10 120 python tools/conv_impls.py --impls 4
    timeout -k 10 120 python tools/conv_impls.py --cin 192 --k 3 1 1 --impls 4
  done
done > $D/conv.txt 2>&1
for v in base ab; do
  if [ $v = ab ]; then export MILNCE_LIB_PATH=$AB; else unset MILNCE_LIB_PATH; fi
  echo "== bench $v"
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 | cut -c1-160
done > $D/bench.txt 2>&1
rm -f $AB
grep -v amdgpu.ids $D/conv.txt $D/bench.txt
