cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r04f; mkdir -p $OUT
for v in "" _kw1 _kw2 "" _kw1 _kw2; do
  SVAE_LIB=$PWD/sparse-vae_amd/sparse_vae/libsvae$v.so timeout -k 10 200 python -u scripts/head_dw_probe.py c2 >> $OUT/probe_c2$v.log 2>&1 || exit $?
done
for v in "" _kw1 _kw2; do
  SVAE_LIB=$PWD/sparse-vae_amd/sparse_vae/libsvae$v.so timeout -k 10 300 python -u scripts/head_dw_probe.py c4 >> $OUT/probe_c4$v.log 2>&1 || exit $?
done
for v in _kw1 _kw2; do
  SVAE_LIB=$PWD/sparse-vae_amd/sparse_vae/libsvae$v.so timeout -k 10 300 python scripts/kw_screen.py 40 > $OUT/screen$v.log 2>&1; rc=$?
  echo "screen $v rc=$rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
