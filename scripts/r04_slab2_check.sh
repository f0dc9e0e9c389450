cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r04u
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_parity_gpu.py -q -rf --timeout 200 --timeout-method thread > gpurun_out/r04u/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/r04u/pytest.log; [ $rc == 0 ] || exit $rc
for i in 1 2; do timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity > gpurun_out/r04u/bench_$i.log 2>&1 || exit $?; tail -1 gpurun_out/r04u/bench_$i.log | cut -c1-160; done
