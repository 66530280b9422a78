cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r2_bisect
mkdir -p $D
for c in 6905c30 2323b00 HEAD; do
  dir=bisect/$c; [ "$c" = HEAD ] && dir=.
  (cd $dir && timeout -k 10 300 python bench.py --steps 2 --warmup 1 --batch_per_gpu 1024 --num_frames 32 --grad_cache_chunks 4 > $GRAFT_REPO_ROOT/$D/c5_$c.log 2>&1) || { echo "c5 $c failed"; tail -5 $D/c5_$c.log; exit 1; }
  echo "c5 $c $(grep -o '"final_loss": [0-9.]*' $D/c5_$c.log) $(grep -o '"ms_per_step": [0-9.]*' $D/c5_$c.log)"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_training.py -k "not learns" -v -s --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
grep -E "embeddings rel|loss on the same|step loss|passed|failed" $D/pytest.log
