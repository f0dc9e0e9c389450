# the 128-tile GEMM's deep ring for small grids: kernel tests + step parity, then C2 / C4 benches alternating
# (SVAE_GEMM_DEEP=0: the 3-stage ring everywhere), then the C2 census with the default
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r04y}; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_parity_gpu.py tests/test_model_gpu.py -q -rf --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; [ $rc == 0 ] || exit $rc
bash scripts/ab_bench.sh ${1:-r04y} "SVAE_GEMM_DEEP=0" "SVAE_GEMM_DEEP=1" "c2 c4" 0 || exit $?
timeout -k 10 300 python -u scripts/gemm_census.py 3 c2 > $OUT/gemm_census_c2.txt 2>&1 || exit $?
