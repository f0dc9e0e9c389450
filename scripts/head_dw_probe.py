"""Where the head dW GEMM's time goes (a_t, b_t, f32 accumulate, M = V, N = d, K = T): plain, with bias row sums,
with k-weighted row sums; each over 20 launches. SVAE_LIB selects the library variant.

    python scripts/head_dw_probe.py [c2|c4]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'sparse-vae_amd'))
import torch  # noqa: E402
from sparse_vae import kernels as K  # noqa: E402
from sparse_vae import _native as N  # noqa: E402

dev = torch.device('cuda', 0)


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else 'c2'
    T, d, V = (32768, 512, 32768) if cfg == 'c2' else (65536, 768, 32768)
    P = (torch.rand(T, V, device=dev) * 0.01).bfloat16()
    hh = torch.randn(T, d, device=dev).bfloat16()
    dW = torch.zeros(V, d, device=dev)
    rs = torch.zeros(V, device=dev)
    kw = torch.rand(T, device=dev)
    slab = torch.empty(2 * V * d, device=dev)
    fl = 2.0 * T * d * V
    cases = {
        'plain': lambda: K.gemm(P, hh, dW, V, d, T, a_t=True, b_t=True, ldb=d, epi=N.EPI_F32_ACC),
        'rowsum': lambda: K.gemm(P, hh, dW, V, d, T, a_t=True, b_t=True, ldb=d, epi=N.EPI_F32_ACC, a_rowsum=rs),
        'k_weight': lambda: K.gemm(P, hh, dW, V, d, T, a_t=True, b_t=True, ldb=d, epi=N.EPI_F32_ACC, a_rowsum=rs,
                                   k_weight=kw),
        'plain_s2': lambda: K.gemm(P, hh, dW, V, d, T, a_t=True, b_t=True, ldb=d, epi=N.EPI_F32_ATOMIC, splits=2),
        'kw_slab2': lambda: K.gemm(P, hh, dW, V, d, T, a_t=True, b_t=True, ldb=d, epi=N.EPI_F32_ATOMIC, splits=2,
                                   aux=slab, a_rowsum=rs, k_weight=kw),
    }
    for r in range(2):
        for name, fn in cases.items():
            ms = timeit(fn)
            print(f'{cfg} head dW M={V} N={d} K={T} {name:9s} {ms * 1e3:8.1f} us {fl / ms / 1e9:7.1f} TF/s', flush=True)


if __name__ == '__main__':
    main()
