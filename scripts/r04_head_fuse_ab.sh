# head backward fusions (the d x GEMM writes the top decoder layer's dropout-masked bf16 gradient; the head LayerNorm
# backward writes bf16(dx * GELU')): kernel tests, step parity, then C2 / C4 benches alternating
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r04hf}; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rf --timeout 200 --timeout-method thread -k "bf16_copy or layernorm or gemm_epilogues or skinny or step_matches or model or eval or dp" > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; [ $rc == 0 ] || exit $rc
bash scripts/ab_bench.sh ${1:-r04hf} "SVAE_HEAD_G2=0 SVAE_LN_GELU=0" "SVAE_HEAD_G2=1 SVAE_LN_GELU=1" "c2 c4" 0 || exit $?
