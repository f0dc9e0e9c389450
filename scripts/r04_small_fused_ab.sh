# token-input prep and step scalars in one launch each: kernel tests, step parity, then C2 / C4 benches alternating
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r04sf}; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rf --timeout 200 --timeout-method thread -k "prep_tokens or step_scalars or step_matches or model or eval or dp or train" > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; [ $rc == 0 ] || exit $rc
bash scripts/ab_bench.sh ${1:-r04sf} "SVAE_SMALL_FUSED=0" "SVAE_SMALL_FUSED=1" "c2 c4" 0 || exit $?
