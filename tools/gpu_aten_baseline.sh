set -e
cd $GRAFT_REPO_ROOT
python -c "import torch; print(torch.cuda.get_device_name(0))"
MILNCE_OPS=aten timeout -k 10 500 python bench.py --steps 3 --warmup 2 --batch_per_gpu 64 > gpurun_out/aten_bs64.json 2> gpurun_out/aten_bs64.err
cat gpurun_out/aten_bs64.json
MILNCE_OPS=aten PYTORCH_MIOPEN_SUGGEST_NHWC=1 timeout -k 10 500 python bench.py --steps 3 --warmup 2 --batch_per_gpu 64 --profile_steps 1 > gpurun_out/aten_nhwc_bs64.json 2> gpurun_out/aten_nhwc_bs64.err
cat gpurun_out/aten_nhwc_bs64.json
