#!/bin/bash
# One PMC pass (COUNTERS, default FETCH_SIZE) over the kernels matching REGEX inside a short C2 bench run.
#   bash scripts/pmc_kernel.sh TAG REGEX [COUNTERS...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/$1
RE=$2
shift 2
CT=${*:-FETCH_SIZE}
mkdir -p "$OUT"
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $CT --kernel-include-regex "$RE" -f csv -d "$OUT/pmc" -o run -- \
  python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-parity > "$OUT/pmc.log" 2>&1
