"""LayerNorm launches of one training step in call order, from a rocprofv3 --kernel-trace directory (verdict r05
item 6: which LayerNorm passes the step runs and what each costs). Prints, for the last full step, every ln_* launch:
kernel, grid, duration; then the totals.   python scripts/ln_census.py gpurun_out/<tag>/prof [steps]
"""
import collections
import csv
import glob
import re
import sys


def main():
    root = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    path = glob.glob(f'{root}/**/*kernel_trace.csv', recursive=True)[0]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r['Start_Timestamp']))
    # a step starts at the embedding forward (one launch per step)
    starts = [i for i, r in enumerate(rows) if 'emb_fwd_kernel' in r['Kernel_Name']]
    if len(starts) < 2:
        print('no step boundaries found')
        return
    a, b = starts[-2], starts[-1]
    tot = collections.defaultdict(float)
    cnt = collections.Counter()
    for r in rows[a:b]:
        name = r['Kernel_Name']
        if not re.search(r'ln_(fwd|bwd)', name):
            continue
        m = re.search(r'(ln_(?:fwd|bwd)\w*?kernel\w*)', name)
        short = m.group(1) if m else name[:60]
        us = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
        grid = int(r['Grid_Size_X']) * int(r.get('Grid_Size_Y', 1) or 1)
        print(f'{short:60s} grid {grid:8d} {us:8.1f} us')
        tot[short] += us
        cnt[short] += 1
    print('--- totals (one step)')
    for k in tot:
        print(f'{k:60s} n={cnt[k]:3d} {tot[k] / 1e3:7.3f} ms')
    print(f'all LayerNorm: {sum(tot.values()) / 1e3:.3f} ms over {sum(cnt.values())} launches')


if __name__ == '__main__':
    main()
