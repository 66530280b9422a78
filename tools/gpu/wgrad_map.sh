# which wgrad kernel each layer's tuner picked (MILNCE_TUNE_LOG) in one bench step
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-wgradmap}
mkdir -p $D
rm -f $D/tune.log
MILNCE_TUNE_LOG=$D/tune.log timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 > $D/bench.log 2>&1
echo "rc=$?"
cat $D/tune.log
