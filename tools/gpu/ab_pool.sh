# Same-box A/B of compile-time options of csrc/pool.hip: bash tools/gpu/ab_pool.sh "FLAGS_A" "FLAGS_B" ...
# Each variant: pool.hip rebuilt with its flags into libmilnce_hip_ab.so (other objects from the
# in-tree build), then tools/ew_bench.py and one bench run; "base" = the in-tree library.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/ab_pool
mkdir -p $D /tmp/abobj
python csrc/build.py > /dev/null
AB=$GRAFT_REPO_ROOT/mil_nce_howto100m_amd/_native/libmilnce_hip_ab.so
: > $D/ew.txt; : > $D/bench.txt
for v in base "$@"; do
  if [ "$v" = base ]; then unset MILNCE_LIB_PATH; else
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -std=c++17 -fPIC -Icsrc -Wno-unused-result -O3 $v -c csrc/pool.hip -o /tmp/abobj/pool.o
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $AB $(ls build/obj/*.o | grep -v /pool.o) /tmp/abobj/pool.o
    export MILNCE_LIB_PATH=$AB
  fi
  echo "== $v" >> $D/ew.txt
  timeout -k 10 200 python tools/ew_bench.py 2>&1 | grep maxpool >> $D/ew.txt
  echo "== $v" >> $D/bench.txt
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>&1 | grep '^{' | cut -c1-160 >> $D/bench.txt
done
rm -f $AB
cat $D/ew.txt $D/bench.txt
