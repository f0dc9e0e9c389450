# k-weight LDS-slot forms with the DMA stagger: screen + timing per form
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r04h}; mkdir -p $OUT
for f in ${2:-1 3}; do
  SVAE_LIB=$PWD/sparse-vae_amd/sparse_vae/libsvae_kw$f.so timeout -k 10 300 python scripts/kw_screen.py 40 > $OUT/screen_kw$f.log 2>&1; rc=$?
  echo "screen kw$f rc=$rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  SVAE_LIB=$PWD/sparse-vae_amd/sparse_vae/libsvae_kw$f.so timeout -k 10 200 python -u scripts/head_dw_probe.py c2 > $OUT/probe_c2_kw$f.log 2>&1 || exit $?
done
