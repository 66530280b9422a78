# BASELINE configs 4 and 5 on one GPU with the current code (soft-DTW loss; 32-frame GradCache step).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --batch_per_gpu 128 --loss sdtw_3 --seq_len 8 > gpurun_out/cfg4_49.json 2> gpurun_out/cfg4_49.err || { tail -30 gpurun_out/cfg4_49.err; exit 1; }
cat gpurun_out/cfg4_49.json
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --batch_per_gpu 1024 --num_frames 32 --grad_cache_chunks 4 > gpurun_out/cfg5_49.json 2> gpurun_out/cfg5_49.err || { tail -30 gpurun_out/cfg5_49.err; exit 1; }
cat gpurun_out/cfg5_49.json
