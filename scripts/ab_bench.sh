#!/bin/bash
# Same-box A/B of bench.py step times: variants alternate (each variant = an env assignment list, e.g.
# "SVAE_LIB=sparse-vae_amd/sparse_vae/libsvae_old.so" or "SVAE_GEMM_STAGGER=0"; "-" = defaults), optionally after a
# GPU test subset run with the default library.
#   TESTS="tests/test_kernels_gpu.py -k 'gemm or attention'" CFGS="c2 c4" ROUNDS=2 bash scripts/ab_bench.sh TAG VARIANT...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-ab}; shift
mkdir -p "$OUT"
if [ -n "${TESTS:-}" ]; then
  eval "timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 150 --timeout-method thread" > "$OUT/tests.log" 2>&1 \
    || { tail -30 "$OUT/tests.log"; exit 1; }
  tail -2 "$OUT/tests.log"
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  for cfg in ${CFGS:-c2}; do
    for v in "$@"; do
      [ "$v" == "-" ] && e="" || e="$v"
      steps=30; [ "$cfg" != c2 ] && steps=10
      line=$(env $e timeout -k 10 300 python -u bench.py --config $cfg --steps $steps --warmup 3 --no-cpu-baseline \
             --no-parity 2>/dev/null | tail -1) || { echo "bench failed: $cfg $v"; exit 1; }
      ms=$(python3 -c "import json,sys; print(json.loads(sys.argv[1])['ms_per_step'])" "$line")
      echo "$cfg [$v] round $r: $ms ms/step" | tee -a "$OUT/ab.log"
    done
  done
done
