#!/bin/bash
# Attention A/B on one box: the attention kernel tests on the in-tree library, then scripts/attn_probe.py
# alternating the in-tree library and sparse_vae/libsvae_aold.so.  bash scripts/attn_ab.sh TAG [PROBE_ONLY]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu --timeout 150 --timeout-method thread -k "attention" > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc = 0 ] || exit $rc
for v in new aold new aold; do
  if [ $v = new ]; then E=SVAE_GEMM_IMPL=0; else E=SVAE_LIB=sparse-vae_amd/sparse_vae/libsvae_$v.so; fi
  env $E ATTN_PROBE_ONLY=${2:-c2c4} timeout -k 10 120 python -u scripts/attn_probe.py > $OUT/attn_$v.txt 2>&1 || exit $?
  echo "== $v"; grep -v amdgpu.ids $OUT/attn_$v.txt
done
