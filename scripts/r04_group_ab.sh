# vocabulary-head forward: tile-row group size of the wide-N GEMM (SVAE_GEMM_GROUP), two passes each, one box
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r04gr}; mkdir -p $OUT
for r in 1 2; do
  for gsz in 4 2 8 16; do
    echo "== group $gsz" >> $OUT/head.log
    SVAE_GEMM_GROUP=$gsz timeout -k 10 200 python -u scripts/head_probe.py >> $OUT/head.log 2>&1 || exit $?
  done
done
