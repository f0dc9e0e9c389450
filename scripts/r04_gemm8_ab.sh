#!/bin/bash
# 8-phase gemm256 (SVAE_GEMM8=1) vs the 2-phase loop on one box: GEMM/engine tests with the 8-phase loop, then
# alternating probe runs of the step's GEMM shapes and of the C2 bench step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-g8}
mkdir -p "$OUT"
SVAE_GEMM8=1 timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_parity_gpu.py -q -x \
  --timeout 150 --timeout-method thread > "$OUT/pytest_g8.log" 2>&1 || { tail -30 "$OUT/pytest_g8.log"; exit 1; }
tail -2 "$OUT/pytest_g8.log"
for r in 1 2; do
  for v in 0 1; do
    SVAE_GEMM8=$v timeout -k 10 300 python scripts/gemm_probe.py all > "$OUT/probe_g8_${v}_$r.log" 2>&1 || exit 1
    echo "== g8=$v run $r"; grep -E "^gemm|^head" "$OUT/probe_g8_${v}_$r.log"
  done
done
for r in 1 2; do
  for v in 0 1; do
    SVAE_GEMM8=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity > "$OUT/bench_g8_${v}_$r.log" 2>&1 || exit 1
    echo "== bench g8=$v run $r"; python -c "import json,sys; d=json.loads(open('$OUT/bench_g8_${v}_$r.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['launch_ms'])"
  done
done
