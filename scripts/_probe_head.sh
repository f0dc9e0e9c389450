set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/head
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_ce_chunked_gpu.py tests/test_engine_parity_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/head/pytest.log 2>&1 && tail -2 gpurun_out/head/pytest.log &&
timeout -k 10 200 python3 -u scripts/head_probe.py > gpurun_out/head/probe.log 2>&1 && cat gpurun_out/head/probe.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/head/prof -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-parity > gpurun_out/head/prof.log 2>&1
rc=$?; tail -1 gpurun_out/head/prof.log; echo rc=$rc; exit $rc
