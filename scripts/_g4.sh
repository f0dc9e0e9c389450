set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/g4
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_ce_chunked_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/g4/pytest_k.log 2>&1; rc=$?; tail -3 gpurun_out/g4/pytest_k.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_engine_parity_gpu.py tests/test_argmax_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/g4/pytest_e.log 2>&1; rc=$?; tail -3 gpurun_out/g4/pytest_e.log; [ $rc = 0 ] || exit $rc
for g in 0 1; do
  echo "== SVAE_GEMM_G4=$g"
  SVAE_GEMM_G4=$g timeout -k 10 200 python3 -u scripts/head_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
  SVAE_GEMM_G4=$g timeout -k 10 200 python3 -u scripts/gemm_probe.py all 2>&1 | grep -v amdgpu.ids | grep gemm || exit 1
  SVAE_GEMM_G4=$g timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity 2>&1 | tail -1 | cut -c1-330 || exit 1
done
