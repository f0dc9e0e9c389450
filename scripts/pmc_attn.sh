#!/bin/bash
# SQ stall breakdown of the attention kernels inside the C2 step (one rocprofv3 --pmc pass, 8 SQ counters).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmc_attn}
mkdir -p "$OUT"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS \
  SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --kernel-include-regex "${2:-attn_(fwd|bwd)_kernel}" \
  -f csv -d "$OUT/pmc" -o run -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-parity > "$OUT/pmc.log" 2>&1
