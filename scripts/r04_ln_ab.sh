# LayerNorm forward: one row per wave (SVAE_LN_FWD_BLOCKS=0) vs rows-per-wave loops with next-row prefetch
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r04n}; mkdir -p $OUT
for c in 0 512 1024 2048 0 1024; do
  SVAE_LN_FWD_BLOCKS=$c timeout -k 10 120 python -u scripts/ln_probe.py >> $OUT/ln_probe.log 2>&1 || exit $?
done
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -k "layernorm or ln_" --timeout 120 --timeout-method thread > $OUT/pytest_ln.log 2>&1; tail -1 $OUT/pytest_ln.log
bash scripts/ab_bench.sh ${1:-r04n} "SVAE_LN_FWD_BLOCKS=0" "SVAE_LN_FWD_BLOCKS=1024" "c2 c4" 0 || exit $?
