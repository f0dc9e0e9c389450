#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r03e
mkdir -p $OUT
ATTN_PROBE_ONLY=c2c4 timeout -k 10 120 python -u scripts/attn_probe.py > $OUT/probe.log 2>&1 || exit $?
cat $OUT/probe.log
bash scripts/ab_bench.sh r03e "SVAE_FUSE_LN=1" "SVAE_FUSE_LN=0" "c4 c2" 1
