# A/B of whole-library GEMM variants in ONE box session: GEMM exactness tests, the vocab-head probe, the C2 shape
# probe (incl. 8K^3 / 4K^3), the bench; for each SVAE_LIB variant ('' = libsvae.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in "$@"; do
  lib=$PWD/sparse-vae_amd/sparse_vae/libsvae${v:+_$v}.so
  echo "== ${v:-current}"
  SVAE_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "gemm or linear_dw" -x -q --timeout 200 --timeout-method thread > gpurun_out/abg_pytest_$v.log 2>&1; rc=$?; tail -1 gpurun_out/abg_pytest_$v.log; [ $rc = 0 ] || exit 1
  SVAE_LIB=$lib timeout -k 10 200 python3 -u scripts/head_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
  SVAE_LIB=$lib timeout -k 10 200 python3 -u scripts/gemm_probe.py all 2>&1 | grep "^gemm" || exit 1
  SVAE_LIB=$lib timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity 2>&1 | tail -1 | cut -c1-200 || exit 1
done
