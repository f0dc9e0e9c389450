# weight-gradient GEMM: split count x implementation (0 = auto, 3 = 256x256, 1 = 128x128 register-staged), with row sums
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for i in 0 3 1; do
  DW_RS=1 SVAE_GEMM_IMPL=$i timeout -k 10 200 python3 -u scripts/dw_split_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
done
