#!/bin/bash
# Round 5: attention probe over several variants on one box (each variant = an env assignment list, e.g.
# "SVAE_ATTN_FWD32=0" or "SVAE_LIB=sparse-vae_amd/sparse_vae/libsvae_fd1.so"), optionally after the attention tests.
#   TESTS=1 PROBE=c2c4 bash scripts/r05_attn_variants.sh TAG VARIANT...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-attn}; shift
mkdir -p "$OUT"
if [ "${TESTS:-1}" == 1 ]; then
  timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "attention" -x -q --timeout 120 \
    --timeout-method thread > "$OUT/attn_tests.log" 2>&1 || { tail -30 "$OUT/attn_tests.log"; exit 1; }
  tail -2 "$OUT/attn_tests.log"
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in "$@"; do
    echo "== $v (round $r)" | tee -a "$OUT/probe.log"
    env $v ATTN_PROBE_ONLY=${PROBE:-c2c4} timeout -k 10 180 python -u scripts/attn_probe.py 2>&1 | grep -v amdgpu.ids | tee -a "$OUT/probe.log" || exit 1
  done
done
