"""Per-GEMM census of a bench config's training step (default C2): every libsvae GEMM launch of a few bench steps
timed with HIP events on its stream, grouped by (M, N, K, layout, epilogue, splits), with TF/s per shape.

    python scripts/gemm_census.py [steps] [config] > profiles/<round>_<config>_gemm_census.txt
"""
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'sparse-vae_amd'))
import torch  # noqa: E402
import bench  # noqa: E402
from sparse_vae import kernels as K  # noqa: E402

EPI = ['bf16', 'f32', 'f32_acc', 'f32_atomic', 'gelu', 'gelu_bwd', 'drop_resid', 'rotary', 'ce_stats', 'ce_prob',
       'rowscale_gather']


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    cfg = sys.argv[2] if len(sys.argv) > 2 else 'c2'
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(0)
    model, opt, sched, batch = bench.build(bench.CONFIGS[cfg], dev)
    print(f'config {cfg}: {bench.CONFIGS[cfg]}')
    for _ in range(3):
        bench.step(model, opt, sched, batch)
    torch.cuda.synchronize()
    rec = []
    orig = K.gemm

    def timed(A, B, C, M, N_, K_, **kw):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        orig(A, B, C, M, N_, K_, **kw)
        e1.record()
        key = (M, N_, K_, int(kw.get('a_t', False)), int(kw.get('b_t', False)), kw.get('epi', 0), kw.get('splits', 1),
               int(kw.get('a_rowsum') is not None), int(kw.get('k_weight') is not None))
        rec.append((key, e0, e1))

    orig_pair = K.gemm_pair

    def timed_pair(g0, g1):   # the paired weight-gradient launch: one record for the two GEMMs (key of both shapes)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        orig_pair(g0, g1)
        e1.record()
        (a0, k0), (a1, k1) = g0, g1
        key = ((a0[3], a1[3]), (a0[4], a1[4]), (a0[5], a1[5]), 1, 1, k0.get('epi', 0), k0.get('splits', 1),
               int(k0.get('a_rowsum') is not None), 0)
        rec.append((key, e0, e1))

    K.gemm = timed
    K.gemm_pair = timed_pair
    for _ in range(steps):
        bench.step(model, opt, sched, batch)
    torch.cuda.synchronize()
    K.gemm = orig
    K.gemm_pair = orig_pair
    agg = defaultdict(lambda: [0, 0.0])
    for key, e0, e1 in rec:
        agg[key][0] += 1
        agg[key][1] += e0.elapsed_time(e1) * 1e3
    total = sum(v[1] for v in agg.values()) / steps
    print(f'GEMM time {total / 1e3:.3f} ms/step (HIP events around each launch, {steps} steps, {cfg} bench step)')
    for key, (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        M, N_, K_, at, bt, epi, sp, rs, kwt = key
        per = us / n
        fl = 2.0 * (sum(a * b * c for a, b, c in zip(M, N_, K_)) if isinstance(M, tuple) else M * N_ * K_)
        print(f'{us / steps / 1e3:7.3f} ms  x{n // steps:2d} {per:9.1f} us {fl / per / 1e6:8.1f} TF/s  '
              f'M={M} N={N_} K={K_} a_t={at} b_t={bt} epi={EPI[epi] if epi < len(EPI) else epi} splits={sp} '
              f'rowsum={rs} k_weight={kwt}')


if __name__ == '__main__':
    main()
