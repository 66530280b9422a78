set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --steps 3 --warmup 3 --profile_steps 1 > gpurun_out/bench34.json 2> gpurun_out/bench34.err || { tail -30 gpurun_out/bench34.err; exit 1; }
cat gpurun_out/bench34.json
wc -l gpurun_out/torch_profile_stacks.txt
