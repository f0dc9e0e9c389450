# round-4 final tree: LayerNorm-forward grid A/B at C2 (same box), then the C4 and C5 bench lines
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r04q}; mkdir -p $OUT
bash scripts/ab_bench.sh ${1:-r04q} "SVAE_LN_FWD_BLOCKS=0" "SVAE_LN_FWD_BLOCKS=1024" "c2" 0 || exit $?
for c in c4 c5; do
  timeout -k 10 400 python -u bench.py --config $c --no-cpu-baseline > $OUT/bench_final_$c.log 2>&1 || exit $?
  tail -1 $OUT/bench_final_$c.log | cut -c1-200
done
