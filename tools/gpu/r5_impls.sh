# per-variant conv timings (cold caches) on the conv_2c / Mixed_3 shapes at bs 256
set -e
cd $GRAFT_REPO_ROOT
D=gpurun_out/${1:-r5impls}
mkdir -p $D
I="4 12 13 14 15 16 17"
{
timeout -k 10 120 python tools/conv_impls.py --cin 64 --cout 192 --k 1 3 3 --t 8 --hw 50 --impls $I --producer 1
timeout -k 10 120 python tools/conv_impls.py --cin 192 --cout 192 --k 3 1 1 --t 8 --hw 50 --impls $I --producer 1
timeout -k 10 120 python tools/conv_impls.py --cin 128 --cout 192 --k 1 3 3 --t 8 --hw 25 --impls $I --producer 1
timeout -k 10 120 python tools/conv_impls.py --cin 96 --cout 128 --k 1 3 3 --t 8 --hw 25 --impls $I --producer 1
} > $D/impls.txt 2>&1
grep -v amdgpu.ids $D/impls.txt
