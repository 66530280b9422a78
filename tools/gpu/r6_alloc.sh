set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r6exp
mkdir -p $D
for e in - PYTORCH_HIP_ALLOC_CONF=expandable_segments:True "PYTORCH_HIP_ALLOC_CONF=expandable_segments:True MILNCE_SIDE_KEEP=1" - ; do
  echo "== config 2 [$e]"
  if [ "$e" = "-" ]; then timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $D/c2.log 2>&1
  else env $e timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $D/c2.log 2>&1; fi
  grep '^{' $D/c2.log | sed -e 's/"metric.*"value": //' -e 's/, "unit.*ms_per_step"/ ms/' -e 's/, "hig.*peak_mem_gib"/ peak/' -e 's/, "plan_hash.*side_stream"/ side/' -e 's/, "kernel_lib.*//'
  grep -i "warn\|expandable" $D/c2.log | head -3 || true
done
