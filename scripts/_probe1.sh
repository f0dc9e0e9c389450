set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/probe1
timeout -k 10 200 python3 -u scripts/gemm_probe.py all > gpurun_out/probe1/gemm_all.log 2>&1 &&
timeout -k 10 200 python3 -u scripts/gemm_probe.py epi > gpurun_out/probe1/gemm_epi.log 2>&1 &&
timeout -k 10 200 python3 -u scripts/attn_probe.py > gpurun_out/probe1/attn.log 2>&1
echo rc=$?
