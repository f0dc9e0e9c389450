# batched LayerNorm-affine column sums: kernel test, step parity + the 2-rank DP test, then C2 / C4 benches alternating
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r04cs}; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rf --timeout 200 --timeout-method thread -k "colsum or step_matches or dp or layernorm or train" > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; [ $rc == 0 ] || exit $rc
bash scripts/ab_bench.sh ${1:-r04cs} "SVAE_COLSUM_BATCH=0" "SVAE_COLSUM_BATCH=1" "c2 c4" 0 || exit $?
