# head dW k-weighted split-K slab form: kernel tests, probe at c4/c2, C4 bench A/B (1 vs 2 splits), C2 bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r04l}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -k "k_weight or rowsum" --timeout 120 --timeout-method thread > $OUT/pytest_kw.log 2>&1 || { tail -20 $OUT/pytest_kw.log; exit 1; }
tail -1 $OUT/pytest_kw.log
timeout -k 10 300 python -u scripts/head_dw_probe.py c4 > $OUT/probe_c4.log 2>&1 || exit $?
timeout -k 10 200 python -u scripts/head_dw_probe.py c2 > $OUT/probe_c2.log 2>&1 || exit $?
bash scripts/ab_bench.sh ${1:-r04l} "SVAE_HEAD_DW_SPLITS=1" "SVAE_HEAD_DW_SPLITS=0" "c4" 0 || exit $?
