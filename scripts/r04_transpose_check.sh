cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r04z; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_parity_gpu.py -q -rf --timeout 200 --timeout-method thread -k "transpose or step_matches" > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; [ $rc == 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-parity > $OUT/prof.log 2>&1 || exit $?
python3 scripts/prof_summary.py $OUT/prof > $OUT/kernel_summary.txt 2>&1
grep -E "kernel time|transpose" $OUT/kernel_summary.txt
rm -rf $OUT/prof
