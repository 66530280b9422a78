# Config-4/5 final-loss bisect over old commits (worktrees under bisect/), then the new tests.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r2_bisect
mkdir -p $D
for c in 6905c30 15b375b 2323b00 HEAD; do
  dir=bisect/$c; [ "$c" = HEAD ] && dir=.
  (cd $dir && timeout -k 10 200 python bench.py --steps 5 --warmup 2 --batch_per_gpu 128 --loss sdtw_3 --seq_len 8 > $GRAFT_REPO_ROOT/$D/c4_$c.log 2>&1) || { echo "c4 $c failed"; tail -5 $D/c4_$c.log; exit 1; }
  echo "c4 $c $(grep -o '"final_loss": [0-9.]*' $D/c4_$c.log) $(grep -o '"ms_per_step": [0-9.]*' $D/c4_$c.log)"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_training.py -k "not learns" -v -s --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
grep -E "embeddings rel|loss on the same|step loss|passed|failed" $D/pytest.log
