# A/B of libsvae builds (SVAE_LIB): GEMM probes + the C2 bench, per variant name ('' = libsvae.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in "$@"; do
  lib=$PWD/sparse-vae_amd/sparse_vae/libsvae${v:+_$v}.so
  echo "== ${v:-current}"
  SVAE_LIB=$lib timeout -k 10 200 python3 -u scripts/head_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
  SVAE_LIB=$lib timeout -k 10 200 python3 -u scripts/gemm_probe.py all 2>&1 | grep -v amdgpu.ids | grep gemm || exit 1
  SVAE_LIB=$lib timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity 2>&1 | tail -1 | cut -c100-200 || exit 1
done
