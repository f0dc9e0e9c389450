#!/bin/bash
# C4 per-rank step: bench line + kernel trace summary, the per-shape GEMM census, and the head-GEMM HBM PMC passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${1:-r04c4}
OUT=gpurun_out/$T
mkdir -p "$OUT"
CFG=c4 bash scripts/gpu_round.sh "$T" bpm || exit $?
timeout -k 10 400 python scripts/gemm_census.py 2 c4 > "$OUT/gemm_census.txt" 2>&1 || exit $?
head -3 "$OUT/gemm_census.txt"
python3 scripts/pmc_head_json.py "$OUT/pmc_fetch" "$OUT/pmc_write" "gemm256_kernel<false, false, 9>" c4 > "$OUT/pmc_head_gemm_c4.json" 2>&1
tail -4 "$OUT/pmc_head_gemm_c4.json"
