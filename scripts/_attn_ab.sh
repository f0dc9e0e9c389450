# A/B of attention builds with scripts/attn_probe.py: args = variant names ('' = libsvae.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/attn_ab
for v in "$@"; do
  lib=sparse-vae_amd/sparse_vae/libsvae${v:+_$v}.so
  echo "== ${v:-current}"
  SVAE_LIB=$PWD/$lib timeout -k 10 200 python3 -u scripts/attn_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
done
