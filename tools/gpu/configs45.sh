# BASELINE configs 4 (soft-DTW SDTW_3, 128 clips) and 5 (32 frames, 1024 clips, 4-way GradCache) on 1 GPU
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/configs45
mkdir -p $D
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --batch_per_gpu 128 --loss sdtw_3 --seq_len 8 > $D/c4.log 2>&1 || { tail -20 $D/c4.log; exit 1; }
grep '^{' $D/c4.log
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --batch_per_gpu 1024 --num_frames 32 --grad_cache_chunks 4 > $D/c5.log 2>&1 || { tail -20 $D/c5.log; exit 1; }
grep '^{' $D/c5.log
