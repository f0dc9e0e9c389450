# GEMM A/B: correctness (GEMM / CE kernel tests, engine parity) and per-shape timing for each variant lib
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/gemm_ab
for v in "$@"; do
  lib=$PWD/sparse-vae_amd/sparse_vae/libsvae${v:+_$v}.so
  echo "== ${v:-current}"
  SVAE_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_ce_chunked_gpu.py tests/test_engine_parity_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gemm_ab/pytest_$v.log 2>&1; rc=$?; tail -1 gpurun_out/gemm_ab/pytest_$v.log; [ $rc = 0 ] || exit $rc
  SVAE_LIB=$lib timeout -k 10 200 python3 -u scripts/gemm_probe.py all 2>&1 | grep -v amdgpu.ids || exit 1
  SVAE_LIB=$lib timeout -k 10 200 python3 -u scripts/gemm_probe.py epi 2>&1 | grep -v amdgpu.ids || exit 1
  SVAE_LIB=$lib timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity 2>&1 | tail -1 | cut -c1-200 || exit 1
done
