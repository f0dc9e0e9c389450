# attention variants: kernel tests + engine parity (incl. the C4 model shape, hd 96) + attn_probe
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/attn_ab4
for v in "$@"; do
  lib=$PWD/sparse-vae_amd/sparse_vae/libsvae${v:+_$v}.so
  echo "== ${v:-current}"
  SVAE_LIB=$lib timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_parity_gpu.py tests/test_argmax_gpu.py -k "attention or parity or oracle or argmax" -x -q --timeout 200 --timeout-method thread > gpurun_out/attn_ab4/pytest_$v.log 2>&1; rc=$?; tail -1 gpurun_out/attn_ab4/pytest_$v.log; [ $rc = 0 ] || exit $rc
  SVAE_LIB=$lib timeout -k 10 200 python3 -u scripts/attn_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
done
