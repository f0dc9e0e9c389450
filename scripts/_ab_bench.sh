# bench-only A/B of whole-library variants in ONE box session, alternating, twice ('' = libsvae.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for rep in 1 2; do
  for v in "$@"; do
    lib=$PWD/sparse-vae_amd/sparse_vae/libsvae${v:+_$v}.so
    echo "== ${v:-current}"
    SVAE_LIB=$lib timeout -k 10 200 python3 -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-parity 2>&1 | tail -1 | cut -c1-200 || exit 1
  done
done
