"""Build profiles/pmc_attention_sq_c2.json from one rocprofv3 --pmc pass of scripts/pmc_attn.sh (8 SQ counters over
the attention kernels of bench.py's C2 step). Each counter is reported as a fraction of SQ_WAVE_CYCLES summed over
the launches of one (kernel, grid) pair.

    python scripts/pmc_attn_json.py gpurun_out/<tag>/pmc "note" > profiles/pmc_attention_sq_c2.json
"""
import collections
import csv
import glob
import json
import re
import sys


def main():
    root, note = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ''
    path = glob.glob(f'{root}/**/*counter_collection.csv', recursive=True)[0]
    sums = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        name = re.sub(r'^void ', '', r['Kernel_Name']).replace('(anonymous namespace)::', '')
        name = re.sub(r'\(.*$', '', name)
        key = f"{name} grid {r.get('Grid_Size', '?')}"
        sums[key][r['Counter_Name']] += float(r['Counter_Value'])
        disp[key].add(r.get('Dispatch_Id', r.get('Correlation_Id', '')))
    out = {'source': 'rocprofv3 --pmc (one pass, 8 SQ counters) on bench.py --steps 3 --warmup 2, scripts/pmc_attn.sh; '
                     'values are fractions of SQ_WAVE_CYCLES. ' + note, 'kernels': {}}
    for key in sorted(sums):
        s = sums[key]
        wc = s.get('SQ_WAVE_CYCLES', 0.0)
        rec = {'launches': len(disp[key]), 'wave_cycles': wc}
        for c in sorted(s):
            if c != 'SQ_WAVE_CYCLES' and wc:
                rec[c] = round(s[c] / wc, 4)
        out['kernels'][key] = rec
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == '__main__':
    main()
