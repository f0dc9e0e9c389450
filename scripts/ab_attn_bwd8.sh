#!/bin/bash
# Attention backward A/B on one box: the 8-wave 256-key kernel (default) vs the 4-wave 128-key kernels
# (SVAE_ATTN_BWD8=0), timed by scripts/attn_probe.py, plus the attention kernel tests and the engine parity.
#   bash scripts/ab_attn_bwd8.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -rf -k "attention" --timeout 150 --timeout-method thread > "$OUT/attn_tests.log" 2>&1; rc=$?
tail -2 "$OUT/attn_tests.log"
[ $rc == 0 ] || exit $rc
timeout -k 10 180 python -u scripts/attn_probe.py > "$OUT/probe_bwd8.log" 2>&1 || exit $?
SVAE_ATTN_BWD8=0 timeout -k 10 180 python -u scripts/attn_probe.py > "$OUT/probe_bwd4.log" 2>&1 || exit $?
timeout -k 10 180 python -u scripts/attn_probe.py > "$OUT/probe_bwd8b.log" 2>&1 || exit $?
cat "$OUT/probe_bwd8.log" "$OUT/probe_bwd4.log" | grep -i "bwd\|fwd" | head -40
timeout -k 10 400 python -u -m pytest tests/test_engine_parity_gpu.py -q -rf --timeout 200 --timeout-method thread > "$OUT/parity.log" 2>&1; rc=$?
tail -2 "$OUT/parity.log"
exit $rc
