set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
# BASELINE config 4 (per-GPU share of bs 1024 on 8 GPUs): soft-DTW SDTW_3 loss over 8-clip sequences
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --batch_per_gpu 128 --loss sdtw_3 --seq_len 8 > gpurun_out/bench_cfg4.json 2> gpurun_out/bench_cfg4.err || { tail -30 gpurun_out/bench_cfg4.err; exit 1; }
cat gpurun_out/bench_cfg4.json
# BASELINE config 5 (per-GPU share of bs 8192 on 8 GPUs): 32 frames, 1024 clips/GPU, GradCache 4 micro-batches
timeout -k 10 900 python bench.py --steps 2 --warmup 1 --batch_per_gpu 1024 --num_frames 32 --grad_cache_chunks 4 > gpurun_out/bench_cfg5.json 2> gpurun_out/bench_cfg5.err || { tail -30 gpurun_out/bench_cfg5.err; exit 1; }
cat gpurun_out/bench_cfg5.json
