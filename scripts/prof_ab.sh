#!/bin/bash
# Kernel-trace profiles of the bench step for two env variants (same box).  bash scripts/prof_ab.sh TAG CFG "ENV_A" "ENV_B"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/$1
CFG=$2
mkdir -p "$OUT"
for v in A B; do
  if [ $v == A ]; then E=$3; else E=$4; fi
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_$v" -o run -- python3 bench.py --config $CFG --steps 10 --warmup 3 --no-cpu-baseline --no-parity > "$OUT/prof_$v.log" 2>&1 || exit $?
  echo "== $v ($E)"; python3 scripts/prof_summary.py "$OUT/prof_$v" | head -30
done
