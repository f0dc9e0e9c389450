# gemm_ov A/B in ONE box session: GEMM + engine tests with SVAE_GEMM_OV=1, then the gemm probe and the bench with
# SVAE_GEMM_OV=0 / 1 alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
SVAE_GEMM_OV=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "gemm or rotary" -x -q --timeout 200 --timeout-method thread > gpurun_out/ov_pytest.log 2>&1; rc=$?; tail -1 gpurun_out/ov_pytest.log; [ $rc = 0 ] || exit 1
SVAE_GEMM_OV=1 timeout -k 10 300 python -u -m pytest tests/test_engine_parity_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ov_pytest2.log 2>&1; rc=$?; tail -1 gpurun_out/ov_pytest2.log; [ $rc = 0 ] || exit 1
for rep in 1 2; do
  for ov in 0 1; do
    echo "== SVAE_GEMM_OV=$ov"
    SVAE_GEMM_OV=$ov timeout -k 10 200 python3 -u scripts/gemm_probe.py epi 2>&1 | grep "^epi" || exit 1
    SVAE_GEMM_OV=$ov timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity 2>&1 | tail -1 | cut -c1-200 || exit 1
  done
done
