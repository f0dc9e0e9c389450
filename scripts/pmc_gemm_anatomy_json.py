"""Reduce scripts/pmc_gemm_anatomy.sh's two passes per gemm256 kernel:

    python scripts/pmc_gemm_anatomy_json.py gpurun_out/<tag> > profiles/pmc_gemm_anatomy_c2.json

SQ_ACTIVE_INST_* and SQ_WAIT_INST_LDS are quad-cycles per wave like SQ_WAVE_CYCLES (fractions of it); SQ_LDS_IDX_ACTIVE,
TA_TA_BUSY, TD_TD_BUSY and the stall counters are summed over the chip's 256 per-CU units, normalised here by the
kernel's active cycles GRBM_GUI_ACTIVE / 8 (GRBM sums the 8 XCDs) x 256 = one unit's busy share (not calibrated against
a known-rate kernel: read them relative to each other)."""
import collections
import csv
import glob
import json
import re
import sys

UNITS = 256


def per_kernel(root):
    path = glob.glob(f'{root}/**/*counter_collection.csv', recursive=True)
    sums = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in (csv.DictReader(open(path[0])) if path else []):
        name = re.sub(r'^void ', '', r['Kernel_Name']).replace('(anonymous namespace)::', '')
        name = re.sub(r'\(.*$', '', name)
        key = f"{name} grid {r.get('Grid_Size', '?')}"
        sums[key][r['Counter_Name']] += float(r['Counter_Value'])
        disp[key].add(r.get('Dispatch_Id') or r.get('Correlation_Id', ''))
    return sums, disp


def main():
    root = sys.argv[1]
    s1, d1 = per_kernel(f'{root}/p1')
    s2, d2 = per_kernel(f'{root}/p2')
    out = {'source': 'rocprofv3 --kernel-trace --pmc, two passes over bench.py --config c2 --steps 2 --warmup 2 '
                     '(scripts/pmc_gemm_anatomy.sh)',
           'units': 'sq_*: fractions of SQ_WAVE_CYCLES; *_busy / *_stall: fraction of the kernel\'s active cycles '
                    'per unit (sum / (GRBM_GUI_ACTIVE / 8 x 32 CUs per XCD))',
           'kernels': {}}
    for key in sorted(set(s1) & set(s2), key=lambda k: -s1[k].get('SQ_WAVE_CYCLES', 0)):
        a, b = s1[key], s2[key]
        wc = a.get('SQ_WAVE_CYCLES', 0.0)
        g1 = a.get('GRBM_GUI_ACTIVE', 0.0) / 8 * UNITS
        g2 = b.get('GRBM_GUI_ACTIVE', 0.0) / 8 * UNITS
        rec = {'launches': len(d1[key])}
        for c in ('SQ_ACTIVE_INST_VMEM', 'SQ_ACTIVE_INST_LDS', 'SQ_ACTIVE_INST_VALU', 'SQ_ACTIVE_INST_SCA',
                  'SQ_ACTIVE_INST_MISC', 'SQ_WAIT_INST_LDS'):
            if wc:
                rec[c.lower()] = round(a.get(c, 0.0) / wc, 4)
        if g1:
            rec['lds_idx_active_busy'] = round(a.get('SQ_LDS_IDX_ACTIVE', 0.0) / g1, 4)
        if g2:
            for c in ('TA_TA_BUSY', 'TA_ADDR_STALLED_BY_TC_CYCLES', 'TD_TD_BUSY', 'TD_TC_STALL',
                      'SQ_VMEM_TA_CMD_FIFO_FULL', 'SQ_VMEM_TA_ADDR_FIFO_FULL', 'SQ_BUSY_CU_CYCLES'):
                rec[c.lower()] = round(b.get(c, 0.0) / g2, 4)
        out['kernels'][key] = rec
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == '__main__':
    main()
