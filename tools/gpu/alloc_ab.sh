# Caching-allocator behaviour under the side-stream wgrads (40 steps, same box): operands kept
# referenced until their event / the drain (MILNCE_SIDE_KEEP=1), until the drain only (2), or
# record_stream'd (0).
cd $GRAFT_REPO_ROOT
D=gpurun_out/${1:-alloc}
mkdir -p $D
f() { grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"peak_mem_gib": [0-9.]*\|"peak_reserved_gib": [0-9.]*' $1 | tr '\n' ' '; echo; }
for r in 1 2; do
  for k in 1 2 0; do
    MILNCE_SIDE_KEEP=$k timeout -k 10 300 python bench.py --steps 40 --warmup 3 > $D/k$k-$r.log 2>&1; echo -n "SIDE_KEEP=$k: "; f $D/k$k-$r.log
  done
done
