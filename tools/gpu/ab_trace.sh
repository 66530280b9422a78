# Same-box A/B of a runtime switch with in-step kernel traces:
#   bash tools/gpu/ab_trace.sh TAG VAR VALUE_A VALUE_B
# bench A B A B, then one rocprofv3 kernel trace per value (kstats per-kernel ms/step).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; VAR=$2; A=$3; B=$4
D=gpurun_out/$TAG
mkdir -p $D
for r in 1 2; do
  for v in "$A" "$B"; do
    echo "== $VAR=$v round $r"
    env $VAR=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 | cut -c1-160
  done
done > $D/bench.txt 2>&1
grep -v amdgpu.ids $D/bench.txt
for arm in a b; do
  if [ $arm = a ]; then v=$A; else v=$B; fi
  # label: the value itself when it is a plain word, else the arm (a / b)
  case "$v" in *[!A-Za-z0-9_.-]*|"") L=$arm ;; *) L=$v ;; esac
  export $VAR=$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof_$L -o run --output-format csv -- python bench.py --steps 3 --warmup 2 > $D/prof_$L.log 2>&1 || { tail -20 $D/prof_$L.log; exit 1; }
  T=$(find $D/prof_$L -name "run_kernel_trace.csv" | head -1)
  python tools/kstats.py $T --skip 3 --top 60 > $D/kstats_$L.txt
  head -3 $D/kstats_$L.txt
done
find $D -name "*.csv" -size +20M -delete
