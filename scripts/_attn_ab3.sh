# correctness (attention kernel tests + engine parity) and attn_probe timing for each variant lib
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/attn_ab3
for v in "$@"; do
  lib=$PWD/sparse-vae_amd/sparse_vae/libsvae${v:+_$v}.so
  echo "== ${v:-current}"
  SVAE_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k attention -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_ab3/pytest_$v.log 2>&1; rc=$?; tail -1 gpurun_out/attn_ab3/pytest_$v.log; [ $rc = 0 ] || exit $rc
  SVAE_LIB=$lib timeout -k 10 200 python3 -u scripts/attn_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
done
