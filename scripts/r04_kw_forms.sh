#!/bin/bash
# Screen the LDS forms of the head dW k-weights (diagnostic builds libsvae_kw{1,2,3}.so, SVAE_KW_FORM) and the
# product (global loads) with scripts/kw_screen.py. A wrong row sum is an ordinary exit 1 (the screen goes on);
# a timeout, abort or fault ends the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-kw}
REPS=${2:-30}
mkdir -p "$OUT"
for f in 0 1 2 3; do
  lib=sparse-vae_amd/sparse_vae/libsvae.so
  [ $f -gt 0 ] && lib=sparse-vae_amd/sparse_vae/libsvae_kw$f.so
  SVAE_LIB=$PWD/$lib timeout -k 10 300 python scripts/kw_screen.py $REPS > "$OUT/kw_form$f.log" 2>&1
  rc=$?
  echo "== form $f rc=$rc"; grep -E "runs|head dW" "$OUT/kw_form$f.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
exit 0
