# per-GEMM split counts in the paired dW launch: kernel tests, step parity, then C2 / C4 benches alternating
# (SVAE_DW_PAIR_EQUAL=1: one common count, the round-3 rule)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r04w}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_parity_gpu.py -q -rf --timeout 200 --timeout-method thread -k "pair or step or rowsum" > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; [ $rc == 0 ] || exit $rc
bash scripts/ab_bench.sh ${1:-r04w} "SVAE_DW_PAIR_EQUAL=1" "SVAE_DW_PAIR_EQUAL=0" "c2 c4" 0 || exit $?
timeout -k 10 300 python -u scripts/gemm_census.py 3 c2 > $OUT/gemm_census_c2.txt 2>&1 || exit $?
