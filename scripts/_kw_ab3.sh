# k-weighted row sums at the use (cur) vs at the end of the K-tile (kwend): exact tests, head dW probe, C2 step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for r in 1 2; do
for v in cur kwend; do
  lib=$PWD/sparse-vae_amd/sparse_vae/libsvae_$v.so
  echo "== $v"
  SVAE_LIB=$lib timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "rowsum" 2>&1 | tail -1 || exit 1
  if [ $r = 1 ]; then SVAE_LIB=$lib timeout -k 10 200 python3 -u scripts/head_probe.py 2>&1 | grep "kw" || exit 1; fi
  SVAE_LIB=$lib timeout -k 10 200 python3 -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-parity 2>&1 | tail -1 | grep -o '"ms_per_step": [0-9.]*' || exit 1
done
done
