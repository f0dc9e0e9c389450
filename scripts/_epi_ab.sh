# A/B of the epilogue operand prefetch depth: stamps (per-tile K-loop / epilogue cycles) for the stamps builds, then
# kernel tests + GEMM probes + bench for each variant (one box session)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=$PWD/sparse-vae_amd/sparse_vae
for v in st0 st42 st84; do
  echo "== stamps $v"
  SVAE_LIB=$L/libsvae_$v.so timeout -k 10 200 python3 -u scripts/gemm_stamps.py 2>&1 | grep -v amdgpu.ids || exit 1
done
bash scripts/_gemm_ab.sh "" "$@"
