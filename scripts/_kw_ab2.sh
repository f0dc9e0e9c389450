# same-box step time: committed build (head) vs the load-at-use k-weights build, alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for r in 1 2; do
for v in head atuse; do
  lib=$PWD/sparse-vae_amd/sparse_vae/libsvae_$v.so
  echo "== $v $(SVAE_LIB=$lib timeout -k 10 200 python3 -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-parity 2>&1 | tail -1 | grep -o '"ms_per_step": [0-9.]*')" || exit 1
done
done
SVAE_LIB=$PWD/sparse-vae_amd/sparse_vae/libsvae_head.so timeout -k 10 200 python3 -u scripts/head_probe.py 2>&1 | grep "kw" || exit 1
