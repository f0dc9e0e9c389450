#!/bin/bash
# GEMM A/B on one box: the GEMM / engine parity tests on the in-tree library, then the C2 step census
# (scripts/gemm_census.py) alternating the in-tree library and sparse_vae/libsvae_old.so.  bash scripts/gemm_ab.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_ce_chunked_gpu.py tests/test_engine_parity_gpu.py -x -q -m gpu --timeout 150 --timeout-method thread -k "gemm or ce_ or prob or c2shape or chunk" > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc = 0 ] || exit $rc
L=sparse-vae_amd/sparse_vae
for v in new old new old; do
  if [ $v = new ]; then E=SVAE_GEMM_IMPL=0; else E=SVAE_LIB=$L/libsvae_$v.so; fi
  env $E timeout -k 10 200 python -u scripts/gemm_census.py 3 > $OUT/census_$v.txt 2>&1 || exit $?
  head -16 $OUT/census_$v.txt
done
