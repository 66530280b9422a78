# box conv ablations (csrc/conv_box.hip BOX_ABLATE), impl 15 on the conv_2c shapes
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-boxabl}
mkdir -p $D /tmp/abobj
python csrc/build.py > /dev/null
for m in ${ABL:-1 2 4 8 15}; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -std=c++17 -fPIC -Icsrc -Wno-unused-result -O3 -DBOX_ABLATE=$m -c csrc/conv_box.hip -o /tmp/abobj/conv_box_$m.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o /tmp/abobj/lib_$m.so $(ls build/obj/*.o | grep -v /conv_box.o) /tmp/abobj/conv_box_$m.o
done
for m in 0 ${ABL:-1 2 4 8 15}; do
  if [ $m = 0 ]; then unset MILNCE_LIB_PATH; else export MILNCE_LIB_PATH=/tmp/abobj/lib_$m.so; fi
  echo "== ablate $m"
  timeout -k 10 120 python tools/conv_impls.py --impls 15
  timeout -k 10 120 python tools/conv_impls.py --cin 192 --k 3 1 1 --impls 15
done > $D/ablate.txt 2>&1
grep -v amdgpu.ids $D/ablate.txt
