# same-box A/B of the attention-backward delta from the dO GEMM epilogue (SVAE_DELTA_FUSED=1) vs its own pass (=0):
# C2 and C4 benches alternating, then a kernel-trace profile of each at C2
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r04j}; mkdir -p $OUT
bash scripts/ab_bench.sh ${1:-r04j} "SVAE_DELTA_FUSED=0" "SVAE_DELTA_FUSED=1" "c2 c4" 0 || exit $?
