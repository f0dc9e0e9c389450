#!/bin/bash
# Vocabulary-head forward epilogue anatomy: the probe on the default library and on diagnostic builds
# (scripts/build_variant.sh NAME gemm.hip -DSVAE_DIAG_NOEXP / -DSVAE_DIAG_NOSTORE).  bash scripts/head_diag.sh TAG VARIANT...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
timeout -k 10 120 python -u scripts/head_probe.py > "$OUT/head_default.txt" 2>&1 || exit $?
for v in "$@"; do
  SVAE_LIB=sparse-vae_amd/sparse_vae/libsvae_$v.so timeout -k 10 120 python -u scripts/head_probe.py > "$OUT/head_$v.txt" 2>&1 || exit $?
done
timeout -k 10 120 python -u scripts/head_probe.py > "$OUT/head_default2.txt" 2>&1 || exit $?
for f in "$OUT"/head_*.txt; do echo "== $f"; head -3 "$f"; done
