# C5 (the C4 model at L = 2048) kernel trace + GEMM census on the final tree
cd "${GRAFT_REPO_ROOT:-/root/repo}"
CFG=c5 bash scripts/gpu_round.sh r04c5 p || exit $?
timeout -k 10 400 python -u scripts/gemm_census.py 2 c5 > gpurun_out/r04c5/gemm_census.txt 2>&1 || exit $?
