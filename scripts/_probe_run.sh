export TMPDIR=/tmp; mkdir -p gpurun_out/gp6
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm or ce_stats" > gpurun_out/gp6/pytest.log 2>&1; rc=$?; tail -15 gpurun_out/gp6/pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_engine_parity_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gp6/pytest2.log 2>&1; rc=$?; tail -3 gpurun_out/gp6/pytest2.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/gp6/bench.log 2>&1; rc=$?; tail -1 gpurun_out/gp6/bench.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/gp6/prof -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-parity > gpurun_out/gp6/prof.log 2>&1
