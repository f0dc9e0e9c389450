# GEMM-only A/B (no tests): per-shape probe + bench, variants alternated twice in one box session
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in "$@"; do
  lib=$PWD/sparse-vae_amd/sparse_vae/libsvae${v:+_$v}.so
  echo "== ${v:-current}"
  SVAE_LIB=$lib timeout -k 10 200 python3 -u scripts/gemm_probe.py all 2>&1 | grep -v "amdgpu.ids\|SVAE_GEMM" || exit 1
  SVAE_LIB=$lib timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity 2>&1 | tail -1 | cut -c1-200 || exit 1
done
