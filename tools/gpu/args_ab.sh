# Same-box comparison of bench.py argument sets (2 rounds each):
# bash tools/gpu/args_ab.sh TAG "ARGS_A" "ARGS_B" ...   ("-" = no extra arguments)
set -e
cd $GRAFT_REPO_ROOT
D=gpurun_out/${1:-argsab}
shift
mkdir -p $D
for r in 1 2; do
  for a in "$@"; do
    echo "== [$a] round $r"
    if [ "$a" = "-" ]; then timeout -k 10 300 python bench.py --steps 20 --warmup 5 | cut -c1-170
    else timeout -k 10 300 python bench.py --steps 20 --warmup 5 $a | cut -c1-170; fi
  done
done > $D/bench.txt 2>&1
grep -v amdgpu.ids $D/bench.txt | sed -e 's/"metric.*"value": //' -e 's/, "unit.*ms_per_step"/ ms/' -e 's/, "hig.*//'
