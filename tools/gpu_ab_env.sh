# A/B one environment toggle on the flagship bench, alternating runs on one box:
#   bash tools/gpu_ab_env.sh VAR   (runs VAR=1, VAR=0, VAR=1, VAR=0)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 1 0 1 0; do
  env $1=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/ab_$1_$v.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }
  echo "$1=$v $(python -c "import json;d=json.load(open('gpurun_out/ab_$1_$v.json'));print(d['ms_per_step'])")"
done
