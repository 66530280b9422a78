set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { tail -80 gpurun_out/pytest_gpu.log; }
tail -5 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --batch_per_gpu 64 > gpurun_out/bench_bs64.json 2> gpurun_out/bench_bs64.err || { tail -30 gpurun_out/bench_bs64.err; exit 1; }
cat gpurun_out/bench_bs64.json
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --batch_per_gpu 256 > gpurun_out/bench_bs256.json 2> gpurun_out/bench_bs256.err || { tail -30 gpurun_out/bench_bs256.err; exit 1; }
cat gpurun_out/bench_bs256.json
