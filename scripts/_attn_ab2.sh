set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attn or attention" --timeout 120 --timeout-method thread 2>&1 | tail -2 &&
timeout -k 10 300 python -u -m pytest tests/test_engine_parity_gpu.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2 &&
bash scripts/_attn_ab.sh base "" base ""
