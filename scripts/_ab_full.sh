# A/B of whole-library variants in ONE box session (box-to-box speed differs by up to ~10 %): kernel tests + engine
# parity, attention probe, head probe, bench, for each SVAE_LIB variant ('' = libsvae.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab_full
for v in "$@"; do
  lib=$PWD/sparse-vae_amd/sparse_vae/libsvae${v:+_$v}.so
  echo "== ${v:-current}"
  SVAE_LIB=$lib timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_parity_gpu.py tests/test_ce_chunked_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_full/pytest_$v.log 2>&1; rc=$?; tail -1 gpurun_out/ab_full/pytest_$v.log; [ $rc = 0 ] || exit $rc
  SVAE_LIB=$lib ATTN_PROBE_ONLY=${ATTN_ONLY:-} timeout -k 10 200 python3 -u scripts/attn_probe.py 2>&1 | grep -v amdgpu.ids | head -3 || exit 1
  SVAE_LIB=$lib timeout -k 10 200 python3 -u scripts/head_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
  SVAE_LIB=$lib timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity 2>&1 | tail -1 | cut -c1-200 || exit 1
done
