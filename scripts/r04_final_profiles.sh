# round-4 final tree: attention SQ counters at C2 (attn_fwd / attn_bwd8), then the C4 kernel trace + GEMM census
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash scripts/pmc_attn.sh r04s_pmc_attn "attn_(fwd|bwd8)_kernel" || exit $?
CFG=c4 bash scripts/gpu_round.sh r04s_c4 p || exit $?
timeout -k 10 300 python -u scripts/gemm_census.py 2 c4 > gpurun_out/r04s_c4/gemm_census.txt 2>&1 || exit $?
