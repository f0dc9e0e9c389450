# the decoder's z-projection forwards in one launch (rows spliced in by each layer's first LayerNorm): kernel tests,
# step parity / model / eval tests, then C2 / C4 benches alternating
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r04zf}; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rf --timeout 200 --timeout-method thread -k "zproj or zsplice or layernorm or step_matches or model or dp or train or eval or argmax or golden" > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; [ $rc == 0 ] || exit $rc
bash scripts/ab_bench.sh ${1:-r04zf} "SVAE_ZPROJ_FWD_BATCH=0" "SVAE_ZPROJ_FWD_BATCH=1" "c2 c4" 0 || exit $?
