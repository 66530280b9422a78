# Config 5 one-shot (1024 clips x 32 frames on one GPU) under several environments:
# bash tools/gpu/c5_env.sh TAG "ENV_A" "ENV_B" ...   ("-" = no extra variables)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-c5env}
shift
mkdir -p $D
i=0
for e in "$@"; do
  i=$((i+1))
  echo "== [$e]"
  if [ "$e" = "-" ]; then timeout -k 10 400 python bench.py --steps 2 --warmup 1 --batch_per_gpu 1024 --num_frames 32 > $D/run$i.log 2>&1
  else env $e timeout -k 10 400 python bench.py --steps 2 --warmup 1 --batch_per_gpu 1024 --num_frames 32 > $D/run$i.log 2>&1; fi
  rc=$?
  grep '^{' $D/run$i.log | sed -e 's/"metric.*"value": //' -e 's/, "unit.*ms_per_step"/ ms/' -e 's/, "hig.*peak_mem_gib"/ peak/' -e 's/, "plan_hash.*//'
  [ $rc -ne 0 ] && { echo "rc=$rc"; tail -3 $D/run$i.log; [ $rc -ge 124 ] && exit 1; }
done
exit 0
