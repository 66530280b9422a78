# BASELINE configs 4 (soft-DTW SDTW_3, 128 clips) and 5 (32 frames, 1024 clips: one-shot step and
# 4-way GradCache) on 1 GPU; each run independent (a one-shot OOM does not stop the others).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-configs45}
mkdir -p $D
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --batch_per_gpu 128 --loss sdtw_3 --seq_len 8 > $D/c4.log 2>&1
echo "config 4 rc=$?"; grep '^{' $D/c4.log | cut -c1-400
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --batch_per_gpu 1024 --num_frames 32 --grad_cache_chunks -1 > $D/c5_oneshot.log 2>&1
rc=$?; echo "config 5 auto (one-shot when it fits) rc=$rc"; grep '^{' $D/c5_oneshot.log | cut -c1-600; [ $rc -ne 0 ] && tail -5 $D/c5_oneshot.log
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --batch_per_gpu 1024 --num_frames 32 --grad_cache_chunks 4 > $D/c5_gc4.log 2>&1
echo "config 5 gradcache-4 rc=$?"; grep '^{' $D/c5_gc4.log | cut -c1-600
exit 0
