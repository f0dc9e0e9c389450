"""Build profiles/pmc_gemm_sq_<cfg>.json / pmc_attention_sq_<cfg>.json from scripts/pmc_gemm_sq.sh passes.

    python scripts/pmc_gemm_sq_json.py gpurun_out/<tag> CFG [gemm|attn] > profiles/pmc_..._CFG.json

Per (kernel, grid): launches, mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8) -- busy SIMD-cycles
over the SIMD-cycles of the dispatches (GRBM_GUI_ACTIVE sums the 8 XCDs' active cycles, MI355X_MICROARCH.md 'DVFS
give-back') -- and the stall fractions of SQ_WAVE_CYCLES (WAIT_ANY: parked at s_waitcnt / barrier; WAIT_INST_ANY: issue
stalls; ACTIVE_INST_ANY: issuing; all three count quad-cycles per wave, so these ratios are consistent). The calibration
pass (8192^3 GEMM, known flops) checks the numerator: MFMA_BUSY x 1024 flop per busy SIMD-cycle (16x16x32: 16384 flop in 16
cycles; 32x32x16: 32768 in 32) must equal 2 M N K per launch; and the denominator: GRBM_GUI_ACTIVE / 8 / duration = the
effective clock (<= 2.4 GHz)."""
import collections
import csv
import glob
import json
import re
import sys

SIMDS = 1024


def rows(root):
    path = glob.glob(f'{root}/**/*counter_collection.csv', recursive=True)
    return list(csv.DictReader(open(path[0]))) if path else []


def durations(root):
    path = glob.glob(f'{root}/**/*kernel_trace.csv', recursive=True)
    d = {}
    for r in (csv.DictReader(open(path[0])) if path else []):
        try:
            d[r.get('Dispatch_Id') or r['Correlation_Id']] = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) * 1e-9
        except (KeyError, ValueError):
            pass
    return d


def per_kernel(root):
    sums = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    dur = durations(root)
    tdur = collections.defaultdict(float)
    for r in rows(root):
        name = re.sub(r'^void ', '', r['Kernel_Name']).replace('(anonymous namespace)::', '')
        name = re.sub(r'\(.*$', '', name)
        key = f"{name} grid {r.get('Grid_Size', '?')}"
        sums[key][r['Counter_Name']] += float(r['Counter_Value'])
        cid = r.get('Dispatch_Id') or r.get('Correlation_Id', '')
        if cid not in disp[key]:
            disp[key].add(cid)
            tdur[key] += dur.get(cid, 0.0)
    return sums, disp, tdur


def record(s, n, t):
    wc = s.get('SQ_WAVE_CYCLES', 0.0)
    grbm = s.get('GRBM_GUI_ACTIVE', 0.0)
    rec = {'launches': n}
    busy = s.get('SQ_VALU_MFMA_BUSY_CYCLES', 0.0)
    if t:
        # busy x 1024 = the MFMA flops (calibrated on the 8K^3 GEMM), over the trace duration at the 2.5 PF peak
        rec['mfma_frac_of_peak'] = round(busy * 1024 / t / 2.5e15, 4)
        rec['us_per_launch'] = round(t / n * 1e6, 1)
    if grbm:
        rec['mfma_util_active_cycles'] = round(busy / (SIMDS * grbm / 8), 4)
        if t:
            rec['effective_clock_ghz'] = round(grbm / 8 / t / 1e9, 3)
    if busy and 'SQ_VALU_MFMA_COEXEC_CYCLES' in s:
        rec['coexec_over_mfma_busy'] = round(s['SQ_VALU_MFMA_COEXEC_CYCLES'] / busy, 4)
    for c in ('SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY', 'SQ_ACTIVE_INST_ANY', 'SQ_LDS_BANK_CONFLICT'):
        if wc and c in s:
            rec[c.lower().replace('sq_', '') + '_frac'] = round(s[c] / wc, 4)
    return rec


def main():
    root, cfg = sys.argv[1], sys.argv[2]
    which = sys.argv[3] if len(sys.argv) > 3 else 'gemm'
    out = {'source': f'rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES '
                     f'SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE (one pass) '
                     f'over bench.py --config {cfg} --steps 3 --warmup 2 (scripts/pmc_gemm_sq.sh)',
           'denominator': 'mfma_frac_of_peak = SQ_VALU_MFMA_BUSY_CYCLES x 1024 flop / (kernel-trace duration x 2.5 PF/s): '
                          'the FLOP-derived fraction of the dense bf16 peak (the calibration pass shows busy x 1024 = '
                          '2 M N K exactly); mfma_util_active_cycles = MFMA_BUSY / (1024 SIMDs x GRBM_GUI_ACTIVE / 8), '
                          'the busy share of the SIMD-cycles at the clock the chip actually ran (GRBM_GUI_ACTIVE also '
                          'counts the profiler gaps around a short dispatch: effective_clock_ghz > 2.4 marks a launch '
                          'where that share is understated); the *_frac fields are fractions of SQ_WAVE_CYCLES '
                          '(quad-cycles per wave, like the WAIT/ACTIVE counters); coexec_over_mfma_busy = '
                          'SQ_VALU_MFMA_COEXEC_CYCLES / MFMA_BUSY (cycles in which vector and matrix instructions '
                          'execute together, per MFMA-busy cycle)'}
    cs, cn, ct = per_kernel(f'{root}/calib')
    for key, s in cs.items():
        n = len(cn[key])
        flops = 2.0 * 8192 ** 3 * n
        busy = s.get('SQ_VALU_MFMA_BUSY_CYCLES', 0.0)
        grbm = s.get('GRBM_GUI_ACTIVE', 0.0)
        cal = {'kernel': key, 'launches': n, 'flops': flops,
               'mfma_busy_x1024_over_flops': round(busy * 1024 / flops, 4) if flops else None,
               'mfma_util_active_cycles': round(busy / (SIMDS * grbm / 8), 4) if grbm else None}
        if ct[key]:
            cal['effective_clock_ghz'] = round(grbm / 8 / ct[key] / 1e9, 3)
            cal['tflops_wall'] = round(flops / ct[key] / 1e12, 1)
            cal['flop_derived_frac_of_peak'] = round(flops / ct[key] / 2.5e15, 4)
            cal['mfma_frac_of_peak_from_counter'] = round(busy * 1024 / ct[key] / 2.5e15, 4)
        out['calibration_8192_cubed'] = cal
    sums, disp, tdur = per_kernel(f'{root}/{cfg}')
    sel = (lambda k: 'gemm' in k) if which == 'gemm' else (lambda k: 'attn' in k)
    recs = {k: record(s, len(disp[k]), tdur[k]) for k, s in sums.items() if sel(k)}
    out['kernels'] = dict(sorted(recs.items(), key=lambda kv: -kv[1].get('us_per_launch', 0) * kv[1]['launches']))
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == '__main__':
    main()
