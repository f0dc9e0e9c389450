set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pab
timeout -k 10 300 python -u -m pytest tests/test_ce_chunked_gpu.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -1 || exit 1
PB="python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-parity"
for v in "" pc; do
  export SVAE_LIB=$PWD/sparse-vae_amd/sparse_vae/libsvae${v:+_$v}.so
  echo "== ${v:-nt}"
  timeout -k 10 200 python3 -u scripts/head_probe.py 2>&1 | grep "fwd CE_PROB" || exit 1
  timeout -k 10 200 $PB 2>&1 | tail -1 | cut -c100-200 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "gemm256_kernel<false, false, 9>" -f csv -d gpurun_out/pab/w_${v:-nt} -o run -- $PB > gpurun_out/pab/w_${v:-nt}.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "gemm256_kernel<false, false, 9>" -f csv -d gpurun_out/pab/f_${v:-nt} -o run -- $PB > gpurun_out/pab/f_${v:-nt}.log 2>&1 || exit 1
done
