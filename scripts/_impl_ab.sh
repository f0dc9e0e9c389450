# A/B of the GEMM implementation choice in the real C2 step: per-shape census with the default dispatch and with
# every GEMM that allows it forced to the 128x128 3-blocks/CU LDS-DMA kernel (SVAE_GEMM_IMPL=2) / register-staged (1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/iab
for i in 0 2 1; do
  SVAE_GEMM_IMPL=$i timeout -k 10 200 python3 -u scripts/gemm_census.py 3 > gpurun_out/iab/census_$i.txt 2>&1 || exit 1
  head -1 gpurun_out/iab/census_$i.txt
done
