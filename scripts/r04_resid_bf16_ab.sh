# bf16 copy from the last decoder layer's dropout + residual epilogue (no [T, d] cast pass): kernel test, step parity,
# then C2 / C4 benches alternating
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r04rb}; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rf --timeout 200 --timeout-method thread -k "dropout_resid or gemm_epilogues or skinny or step_matches or model or eval" > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; [ $rc == 0 ] || exit $rc
bash scripts/ab_bench.sh ${1:-r04rb} "SVAE_RESID_BF16=0" "SVAE_RESID_BF16=1" "c2 c4" 0 || exit $?
