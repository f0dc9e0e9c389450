set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/census
timeout -k 10 200 python3 -u scripts/gemm_census.py 3 > gpurun_out/census/gemm_census.txt 2>&1 &&
timeout -k 10 300 python3 -u bench.py --config c4 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/census/bench_c4.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py --config c5 --steps 6 --warmup 2 --no-cpu-baseline --no-parity > gpurun_out/census/bench_c5.log 2>&1
rc=$?; echo rc=$rc; exit $rc
