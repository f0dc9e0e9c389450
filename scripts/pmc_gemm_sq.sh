#!/bin/bash
# SQ counters of the GEMM and attention kernels with a calibrated denominator (verdict r04 item 4). One rocprofv3 --pmc
# pass each (7 SQ counters + GRBM_GUI_ACTIVE; a pass holds at most 8 SQ counters):
#   calib : scripts/gemm_calib.py (8192^3 bf16 GEMM, 7 launches): SQ_VALU_MFMA_BUSY_CYCLES x 1024 flop / busy SIMD-cycle
#           is checked against the GEMM's 2 M N K flops, and GRBM_GUI_ACTIVE / 8 (the per-XCD active cycles) against the
#           kernel-trace duration x clock, so MFMA utilisation = MFMA_BUSY / (1024 SIMDs x GRBM_GUI_ACTIVE / 8);
#   c2/c4 : the same counters over bench.py's step (--steps 3 --warmup 2), kernels matching gemm256|attn_.
#   bash scripts/pmc_gemm_sq.sh TAG [calib c2 c4]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmc_sq}
shift
mkdir -p "$OUT"
CT="SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
for what in ${*:-calib c2 c4}; do
  if [ "$what" == calib ]; then
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CT --kernel-include-regex gemm256 -f csv -d "$OUT/calib" -o run -- \
      python3 scripts/gemm_calib.py > "$OUT/calib.log" 2>&1 || exit 1
  else
    timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $CT --kernel-include-regex "gemm256|attn_" -f csv -d "$OUT/$what" \
      -o run -- python3 bench.py --config $what --steps 3 --warmup 2 --no-cpu-baseline --no-parity > "$OUT/$what.log" 2>&1 || exit 1
  fi
  echo "pmc $what done"
done
