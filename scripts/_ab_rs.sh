# A/B of the bias-gradient row sums (VALU vs MFMA): GEMM / CE kernel tests, head probe, dW split probe, bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab_rs
for v in "$@"; do
  lib=$PWD/sparse-vae_amd/sparse_vae/libsvae${v:+_$v}.so
  echo "== ${v:-current}"
  SVAE_LIB=$lib timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_ce_chunked_gpu.py tests/test_engine_parity_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_rs/pytest_$v.log 2>&1; rc=$?; tail -1 gpurun_out/ab_rs/pytest_$v.log; [ $rc = 0 ] || exit $rc
  SVAE_LIB=$lib timeout -k 10 200 python3 -u scripts/head_probe.py 2>&1 | grep "dW" || exit 1
  SVAE_LIB=$lib timeout -k 10 200 python3 -u scripts/dw_split_probe.py 2>&1 | grep auto || exit 1
  SVAE_LIB=$lib timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity 2>&1 | tail -1 | cut -c1-200 || exit 1
done
