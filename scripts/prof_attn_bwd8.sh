#!/bin/bash
# Kernel-level split (rocprofv3 --kernel-trace --stats) of the attention probe at the C2 and C4 decoder shapes, for the
# 8-wave backward (default) and the 4-wave one (SVAE_ATTN_BWD8=0).   bash scripts/prof_attn_bwd8.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p "$OUT"
ATTN_PROBE_ONLY=c2c4 timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/p8" -o run -- python3 scripts/attn_probe.py > "$OUT/p8.log" 2>&1 || exit $?
ATTN_PROBE_ONLY=c2c4 SVAE_ATTN_BWD8=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/p4" -o run -- python3 scripts/attn_probe.py > "$OUT/p4.log" 2>&1 || exit $?
for v in p8 p4; do echo "== $v"; grep -h "^B=" "$OUT/$v.log"; python3 - "$OUT/$v" <<'PY'
import csv, glob, sys
path = glob.glob(sys.argv[1] + '/**/*kernel_trace.csv', recursive=True)[0]
agg = {}
for r in csv.DictReader(open(path)):
    k = (r['Kernel_Name'][:60], r['Grid_Size_X'] if 'Grid_Size_X' in r else r.get('Grid_Size', ''))
    a = agg.setdefault(k, [0, 0.0])
    a[0] += 1
    a[1] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
for k, (n, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
    if 'attn' in k[0]:
        print(f'{t / n:9.1f} us  n={n:4d}  {k[0]}  grid={k[1]}')
PY
done
