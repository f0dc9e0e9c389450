#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r03o; mkdir -p $OUT
bash scripts/gemm_ab.sh r03o || exit $?
for v in default afwd4 default afwd4; do
  if [ $v = default ]; then E=SVAE_GEMM_IMPL=0; else E=SVAE_LIB=sparse-vae_amd/sparse_vae/libsvae_$v.so; fi
  env $E ATTN_PROBE_ONLY=c2c4 timeout -k 10 120 python -u scripts/attn_probe.py > $OUT/attn_$v.txt 2>&1 || exit $?
  echo "== $v"; grep -v amdgpu.ids $OUT/attn_$v.txt
done
