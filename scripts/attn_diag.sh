#!/bin/bash
# Attention diagnostics on one GPU box: the forward's per-block cycle anatomy (stamps build, C2 decoder shape), the
# kernel probe (C2 and C4 decoder shapes), SQ counter passes over the attention kernels inside the C2 and C4 steps,
# and a C4 kernel trace. Every GPU step has its own time limit; the chain stops at the first failure.
#   bash scripts/attn_diag.sh TAG [STAGES]    STAGES: any of s(tamps) a(probe) q(SQ c2) Q(SQ c4) k(C4 trace)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-attn_diag}
ST=${2:-saqQk}
mkdir -p "$OUT"
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES"
RE='attn_(fwd|bwd8?)_kernel'
rc=0
if [[ $ST == *s* && $rc == 0 ]]; then
  SVAE_LIB=sparse-vae_amd/sparse_vae/libsvae_stamps.so timeout -k 10 180 python3 -u scripts/attn_stamps.py \
    > "$OUT/stamps.log" 2>&1; rc=$?
  tail -12 "$OUT/stamps.log"
fi
if [[ $ST == *a* && $rc == 0 ]]; then
  ATTN_PROBE_ONLY=c2c4 timeout -k 10 180 python3 -u scripts/attn_probe.py > "$OUT/probe.log" 2>&1; rc=$?
  tail -4 "$OUT/probe.log"
fi
if [[ $ST == *q* && $rc == 0 ]]; then
  timeout -s KILL 150 rocprofv3 --pmc $SQ --kernel-include-regex "$RE" -f csv -d "$OUT/sq_c2" -o run -- \
    python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-parity > "$OUT/sq_c2.log" 2>&1; rc=$?
fi
if [[ $ST == *Q* && $rc == 0 ]]; then
  timeout -s KILL 240 rocprofv3 --pmc $SQ --kernel-include-regex "$RE" -f csv -d "$OUT/sq_c4" -o run -- \
    python3 bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline --no-parity > "$OUT/sq_c4.log" 2>&1; rc=$?
fi
if [[ $ST == *k* && $rc == 0 ]]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_c4" -o run -- \
    python3 bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-parity > "$OUT/prof_c4.log" 2>&1; rc=$?
  tail -1 "$OUT/prof_c4.log"
fi
find "$OUT" -type f -size +8M -print -delete
echo "attn_diag rc=$rc"
exit $rc
