# v4 conv main-loop ablations (csrc/conv_v4.hip V4_ABLATE): builds one library per mask and
# times impl 12 / 13 of the conv_2c shapes with each. bash tools/gpu/v4_ablate.sh TAG
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-v4abl}
mkdir -p $D /tmp/abobj
python csrc/build.py > /dev/null
for m in 1 2 3 4 7; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -std=c++17 -fPIC -Icsrc -Wno-unused-result -O3 -DV4_ABLATE=$m -c csrc/conv_v4.hip -o /tmp/abobj/conv_v4_$m.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o /tmp/abobj/lib_$m.so $(ls build/obj/*.o | grep -v /conv_v4.o) /tmp/abobj/conv_v4_$m.o
done
for m in 0 1 2 3 4 7; do
  if [ $m = 0 ]; then unset MILNCE_LIB_PATH; else export MILNCE_LIB_PATH=/tmp/abobj/lib_$m.so; fi
  echo "== ablate $m"
  timeout -k 10 120 python tools/conv_impls.py --impls 12 13
  timeout -k 10 120 python tools/conv_impls.py --cin 192 --k 3 1 1 --impls 12 13
  timeout -k 10 120 python tools/conv_impls.py --cin 128 --cout 192 --hw 25 --impls 12 13
done > $D/ablate.txt 2>&1
grep -v amdgpu.ids $D/ablate.txt
