# Side-stream memory: config 2 peak reserved under record_stream vs kept references (MILNCE_SIDE_KEEP=1),
# then config 5 one-shot inline vs side stream with kept references.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-r6mem}
mkdir -p $D
for e in - MILNCE_SIDE_KEEP=1 MILNCE_SIDE_KEEP=2; do
  echo "== config 2 [$e]"
  if [ "$e" = "-" ]; then timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $D/c2.log 2>&1
  else env $e timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $D/c2.log 2>&1; fi
  grep '^{' $D/c2.log | sed -e 's/"metric.*"value": //' -e 's/, "unit.*ms_per_step"/ ms/' -e 's/, "hig.*peak_mem_gib"/ peak/' -e 's/, "plan_hash.*side_stream"/ side/' -e 's/, "kernel_lib.*//'
done
bash tools/gpu/c5_env.sh $1_c5 - "MILNCE_WGRAD_SIDE_MEM_FRAC=0.95 MILNCE_SIDE_KEEP=1" "MILNCE_WGRAD_SIDE_MEM_FRAC=0.95"
