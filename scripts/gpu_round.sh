#!/bin/bash
# One GPU-box pass: GPU tests, the default bench line, a kernel-trace profile and the two HBM PMC passes
# for the vocab-head GEMM. Every GPU step has its own time limit; the chain stops at the first failure.
#   bash scripts/gpu_round.sh TAG [STAGES]     STAGES: any of t(ests) b(ench) p(rofile) m(pmc); default tbpm
#   CFG=c4 bash scripts/gpu_round.sh ...        bench / profile / PMC on another bench.py config (default c2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-run}
ST=${2:-tbpm}
mkdir -p "$OUT"
HEAD_RE="gemm256_kernel<false, false, 9>"
CFG=${CFG:-c2}
PB="python3 bench.py --config $CFG --steps 10 --warmup 3 --no-cpu-baseline --no-parity"
run() { echo "== $*" >&2; "$@"; }
rc=0
if [[ $ST == *t* && $rc == 0 ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --maxfail=10 --timeout 150 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
  tail -3 "$OUT/pytest_gpu.log"
fi
if [[ $ST == *b* && $rc == 0 ]]; then
  timeout -k 10 300 python -u bench.py --config $CFG > "$OUT/bench.log" 2>&1; rc=$?
  tail -1 "$OUT/bench.log"
fi
if [[ $ST == *p* && $rc == 0 ]]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof" -o run -- $PB > "$OUT/prof.log" 2>&1; rc=$?
  tail -1 "$OUT/prof.log"
  # the per-step summary and the --stats table are small; the trace itself is dropped below (> 8 MB)
  [ $rc == 0 ] && python3 scripts/prof_summary.py "$OUT/prof" > "$OUT/kernel_summary.txt" 2>&1
  [ $rc == 0 ] && python3 scripts/ln_census.py "$OUT/prof" > "$OUT/ln_census.txt" 2>&1
  find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
fi
if [[ $ST == *m* && $rc == 0 ]]; then
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$HEAD_RE" -f csv -d "$OUT/pmc_fetch" -o run -- $PB > "$OUT/pmc_fetch.log" 2>&1; rc=$?
fi
if [[ $ST == *m* && $rc == 0 ]]; then
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$HEAD_RE" -f csv -d "$OUT/pmc_write" -o run -- $PB > "$OUT/pmc_write.log" 2>&1; rc=$?
fi
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; tail -1 "$OUT/smoke.log"
find "$OUT" -type f -size +8M -print -delete
echo "gpu_round rc=$rc"
exit $rc
