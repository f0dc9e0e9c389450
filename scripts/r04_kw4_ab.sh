# k-weight form 4 (register prefetch ahead of the DMA pieces, libsvae_kw4.so): race screen + head-dW timing for forms
# 0 and 4, the k-weight GEMM tests and step parity on form 4, then C2 / C4 benches alternating the two libraries
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r04kw4}; mkdir -p $OUT
L4=$PWD/sparse-vae_amd/sparse_vae/libsvae_kw4.so
L0=$PWD/sparse-vae_amd/sparse_vae/libsvae.so
SVAE_LIB=$L0 timeout -k 10 300 python scripts/kw_screen.py 10 > $OUT/kw_form0.log 2>&1; rc=$?
echo "== form 0 rc=$rc"; grep -E "runs|head dW" $OUT/kw_form0.log; [ $rc -le 1 ] || exit $rc
SVAE_LIB=$L4 timeout -k 10 300 python scripts/kw_screen.py 10 > $OUT/kw_form4.log 2>&1; rc=$?
echo "== form 4 rc=$rc"; grep -E "runs|head dW" $OUT/kw_form4.log; [ $rc == 0 ] || exit $rc
SVAE_LIB=$L4 timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 200 --timeout-method thread -k "k_weight or head or step_matches or ce_chunked" > $OUT/pytest_kw4.log 2>&1; rc=$?
tail -2 $OUT/pytest_kw4.log; [ $rc == 0 ] || exit $rc
bash scripts/ab_bench.sh ${1:-r04kw4} "SVAE_LIB=$L0" "SVAE_LIB=$L4" "c2 c4" 0 || exit $?
