set -e
cd $GRAFT_REPO_ROOT
D=gpurun_out/${1:-r5fused}
mkdir -p $D
{
timeout -k 10 120 python tools/box_fused_bench.py --cin 64 --cout 192 --k 1 3 3 --t 8 --hw 50
timeout -k 10 120 python tools/box_fused_bench.py --cin 192 --cout 192 --k 3 1 1 --t 8 --hw 50
timeout -k 10 120 python tools/box_fused_bench.py --cin 128 --cout 192 --k 1 3 3 --t 8 --hw 25
timeout -k 10 120 python tools/box_fused_bench.py --cin 96 --cout 128 --k 1 3 3 --t 8 --hw 25
timeout -k 10 120 python tools/box_fused_bench.py --cin 192 --cout 192 --k 3 1 1 --t 8 --hw 25
} > $D/fused.txt 2>&1
grep -v amdgpu.ids $D/fused.txt
