# Paired weight-gradient launches: kernel tests + engine parity, then bench with SVAE_DW_PAIR=0 / 1 alternating
# (one box session)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/dwpair
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_parity_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/dwpair/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/dwpair/pytest.log; [ $rc = 0 ] || exit $rc
for v in 0 1 0 1; do
  echo "== SVAE_DW_PAIR=$v"
  SVAE_DW_PAIR=$v timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity 2>&1 | tail -1 | cut -c1-200 || exit 1
done
