"""Per-step kernel time summary of a rocprofv3 --kernel-trace run of bench.py.

    python scripts/prof_summary.py gpurun_out/<tag>/prof [steps]

Groups dispatches by (kernel name, grid size); times are averaged per step over the last `steps` steps
(default: 10, the profiled bench's --steps), which excludes warmup by keeping only the tail of the trace.
"""
import csv
import glob
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    path = glob.glob(f'{root}/**/*kernel_trace.csv', recursive=True)[0]
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    # the RAdam kernel runs once per step: use it to find step boundaries
    marks = [i for i, r in enumerate(rows) if 'radam_kernel' in r['Kernel_Name']]
    if len(marks) > steps:
        rows = rows[marks[-steps - 1] + 1: marks[-1] + 1]
    agg = defaultdict(lambda: [0, 0.0])
    for r in rows:
        name = r['Kernel_Name'].replace('(anonymous namespace)::', '').split('(')[0][:70]
        key = (name, r['Grid_Size'] if 'Grid_Size' in r else r.get('Grid_Size_X', ''))
        agg[key][0] += 1
        agg[key][1] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6
    total = sum(v[1] for v in agg.values()) / steps
    span = (int(rows[-1]['End_Timestamp']) - int(rows[0]['Start_Timestamp'])) / 1e6 / steps
    print(f'kernel time {total:.3f} ms/step, wall span {span:.3f} ms/step over {steps} steps')
    for (name, grid), (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f'{t / steps:8.3f} ms/step {100 * t / steps / total:5.1f}%  n/step={n / steps:5.1f} '
              f'avg {1e3 * t / n:8.1f} us  grid={grid:>9}  {name}')


if __name__ == '__main__':
    main()
