# k-weighted row sums: exact test x3 and head/bench timing for the register-prefetch build and the load-at-use build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/kw
for v in "" atuse; do
  lib=$PWD/sparse-vae_amd/sparse_vae/libsvae${v:+_$v}.so
  echo "== ${v:-prefetch}"
  for i in 1 2 3; do
    SVAE_LIB=$lib timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "rowsum" 2>&1 | tail -1 || exit 1
  done
  SVAE_LIB=$lib timeout -k 10 200 python3 -u scripts/head_probe.py 2>&1 | grep "kw" || exit 1
  SVAE_LIB=$lib timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity 2>&1 | tail -1 | grep -o '"ms_per_step": [0-9.]*' || exit 1
done
