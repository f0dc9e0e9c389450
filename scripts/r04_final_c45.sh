# final round-4 tree: the C4 and C5 bench lines (each with its parity and CPU-baseline legs)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r04f}; mkdir -p $OUT
timeout -k 10 400 python -u bench.py --config c4 > $OUT/bench_c4.log 2>&1 || exit $?
tail -1 $OUT/bench_c4.log | cut -c1-300
timeout -k 10 400 python -u bench.py --config c5 > $OUT/bench_c5.log 2>&1 || exit $?
tail -1 $OUT/bench_c5.log | cut -c1-300
