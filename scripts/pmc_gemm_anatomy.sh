#!/bin/bash
# Where the gemm256 K loop spends its issue and its memory pipe: two rocprofv3 --pmc passes over bench.py's C2 step
# (kernels matching gemm256), one of SQ instruction-class activity, one of the TA / TD (vector-memory address and data)
# pipes; scripts/pmc_gemm_anatomy_json.py reduces them per kernel.
#   bash scripts/pmc_gemm_anatomy.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmc_anat}
mkdir -p "$OUT"
P1="SQ_WAVE_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
P2="TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TD_TD_BUSY TD_TC_STALL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE"
i=0
for CT in "$P1" "$P2"; do
  i=$((i + 1))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $CT --kernel-include-regex "gemm256" -f csv -d "$OUT/p$i" -o run -- \
    python3 bench.py --config c2 --steps 2 --warmup 2 --no-cpu-baseline --no-parity > "$OUT/p$i.log" 2>&1 || exit 1
  echo "pass $i done"
done
