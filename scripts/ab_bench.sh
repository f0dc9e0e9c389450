#!/bin/bash
# Same-box A/B of an engine switch: GPU tests once, then the bench alternating the variants.
#   bash scripts/ab_bench.sh TAG "ENV_A" "ENV_B" [CONFIGS] [TESTS]   e.g. ab_bench.sh r03d "SVAE_FUSE_LN=1" "SVAE_FUSE_LN=0" "c2 c4" 1
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1
A=$2
B=$3
CFGS=${4:-c2}
mkdir -p "$OUT"
if [ "${5:-1}" == 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --maxfail=10 --timeout 200 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
  tail -3 "$OUT/pytest_gpu.log"
  [ $rc == 0 ] || exit $rc
fi
for cfg in $CFGS; do
  for v in A B A B; do
    eval "E=\$$v"
    env $E timeout -k 10 300 python -u bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline --no-parity > "$OUT/bench_${cfg}_$v.log" 2>&1 || exit $?
    echo "$cfg $v ($E): $(tail -1 "$OUT/bench_${cfg}_$v.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], "ms/step", d["value"], "tok/s")')"
  done
done
