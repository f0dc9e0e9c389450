# the decoder's z-projection backwards in one launch: kernel test, step parity + DP tests, then C2 / C4 benches alternating
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r04zp}; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rf --timeout 200 --timeout-method thread -k "zproj or step_matches or model or dp or train or eval" > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; [ $rc == 0 ] || exit $rc
bash scripts/ab_bench.sh ${1:-r04zp} "SVAE_ZPROJ_BATCH=0" "SVAE_ZPROJ_BATCH=1" "c2 c4" 0 || exit $?
