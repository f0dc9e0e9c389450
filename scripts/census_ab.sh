#!/bin/bash
# GEMM census of the C2 step under two env variants (same box).  bash scripts/census_ab.sh TAG "ENV_A" "ENV_B"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1
mkdir -p "$OUT"
env $2 timeout -k 10 200 python -u scripts/gemm_census.py 3 > "$OUT/census_A.txt" 2>&1 || exit $?
env $3 timeout -k 10 200 python -u scripts/gemm_census.py 3 > "$OUT/census_B.txt" 2>&1 || exit $?
head -22 "$OUT/census_A.txt"; echo; head -22 "$OUT/census_B.txt"
