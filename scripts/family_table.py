"""Kernel time per training step by kernel family, from a scripts/prof_summary.py table (kernel_summary.txt of a
`rocprofv3 --kernel-trace --stats` run of bench.py): the one-screen current-state view of DESIGN.md §6.

    python scripts/family_table.py profiles/<tag>_kernel_summary.txt
"""
import re
import sys

# (family, bound, regex over the kernel name); first match wins
FAMILIES = [
    ('vocab head GEMMs (fwd CE_PROB, dX, k-weighted dW)', 'MFMA',
     r'gemm256_kernel<(false, false, (9|10)|true, true, (64|66))>'),
    ('weight-gradient GEMMs (paired split-K) + slab reduce', 'MFMA', r'gemm256_pair_kernel|gemm256_kernel<true, true, 67>|slab_reduce'),
    ('forward / dX GEMMs (fused epilogues)', 'MFMA', r'gemm256_kernel|gemm_glds_kernel|gemm_kernel|gemm_skinny'),
    ('attention backward (+ dQ reduce, delta, [CLS] split)', 'MFMA / sync',
     r'attn_bwd|attn_dq_reduce|attn_delta|attn_cls'),
    ('attention forward (+ split-KV combine)', 'MFMA', r'attn_fwd'),
    ('LayerNorm (fwd, bwd, affine column sums)', 'HBM', r'ln_fwd|ln_bwd|colsum|resid_ln'),
    ('clip + RAdam (norm, update)', 'HBM', r'radam|sumsq|clip_scale'),
    ('embedding, CE rows, z projections, reparam, misc', 'HBM / latency', r'.'),
]


def main():
    path = sys.argv[1]
    total = None
    fam = {f[0]: [0.0, 0] for f in FAMILIES}
    for line in open(path):
        m = re.match(r'kernel time ([\d.]+) ms/step', line)
        if m:
            total = float(m.group(1))
            continue
        m = re.match(r'\s*([\d.]+) ms/step\s+[\d.]+%\s+n/step=\s*([\d.]+).*grid=\s*\d+\s+(.*)$', line)
        if not m:
            continue
        ms, n, name = float(m.group(1)), float(m.group(2)), m.group(3)
        for f, _, rx in FAMILIES:
            if re.search(rx, name):
                fam[f][0] += ms
                fam[f][1] += n
                break
    print(f'kernel time {total:.3f} ms/step ({path})')
    print('| family | ms/step | share | launches/step | bound |')
    print('|---|---|---|---|---|')
    for f, b, _ in FAMILIES:
        ms, n = fam[f]
        print(f'| {f} | {ms:.2f} | {100 * ms / total:.1f} % | {n:.0f} | {b} |')


if __name__ == '__main__':
    main()
