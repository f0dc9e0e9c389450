"""Race screen + timing of the k-weighted bias row sums of the head dW GEMM (gemm256 ACC_KW).

    python scripts/kw_screen.py [reps]

Runs the a_t GEMM with f32 accumulate and k-weighted row sums on integer data (exact in f32) `reps` times per shape
and counts row sums that differ from the exact reference; then times the C2 head-dW shape (32768 x 512 x 32768,
MN-contiguous B) over 20 launches. SVAE_LIB selects the library variant.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'sparse-vae_amd'))
import torch  # noqa: E402
from sparse_vae import kernels as K  # noqa: E402
from sparse_vae import _native as N  # noqa: E402

dev = torch.device('cuda', 0)


def screen(reps):
    g = torch.Generator(device=dev).manual_seed(5)
    total_bad = 0
    for (Kk, M, Nn, b_t) in [(2048, 16384, 776, True), (2048, 16384, 776, False), (32768, 4096, 512, True),
                             (4160, 8192, 1024, True)]:
        A = torch.randint(-2, 3, (Kk, M), device=dev, generator=g).float()
        B = torch.randint(-2, 3, (Kk, Nn), device=dev, generator=g).float()
        kw = torch.randint(-2, 3, (Kk,), device=dev, generator=g).float()
        Bs = (B if b_t else B.t().contiguous()).bfloat16()
        Ab = A.bfloat16()
        ref = 3 + (A * kw[:, None]).sum(0)
        ref_c = 1 + A.t() @ B
        bad_runs, bad_rows, c_bad = 0, 0, 0
        for r in range(reps):
            C = torch.ones(M, Nn, device=dev)
            rs = torch.full((M,), 3.0, device=dev)
            K.gemm(Ab, Bs, C, M, Nn, Kk, a_t=True, b_t=b_t, ldb=Nn if b_t else Kk, epi=N.EPI_F32_ACC, a_rowsum=rs,
                   k_weight=kw)
            torch.cuda.synchronize()
            nb = int((rs != ref).sum())
            bad_rows += nb
            bad_runs += nb > 0
            if r < 3:
                c_bad += int(not torch.equal(C, ref_c))
        total_bad += bad_runs + c_bad
        print(f'K={Kk} M={M} N={Nn} b_t={b_t}: {reps} runs, {bad_runs} with wrong row sums ({bad_rows} rows), '
              f'C wrong in {c_bad} of 3', flush=True)
    return total_bad


def timing():
    T, d, V = 32768, 512, 32768
    P = (torch.rand(T, V, device=dev) * 0.01).bfloat16()
    hh = torch.randn(T, d, device=dev).bfloat16()
    dW = torch.zeros(V, d, device=dev)
    rs = torch.zeros(V, device=dev)
    kw = torch.rand(T, device=dev)
    fn = lambda: K.gemm(P, hh, dW, V, d, T, a_t=True, b_t=True, ldb=d, epi=N.EPI_F32_ACC, a_rowsum=rs, k_weight=kw)
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    print(f'head dW M={V} N={d} K={T} k-weighted: {ms * 1e3:.1f} us  {2.0 * T * d * V / ms / 1e9:.1f} TF/s', flush=True)


if __name__ == '__main__':
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    print('lib', os.environ.get('SVAE_LIB', 'libsvae.so'))
    bad = screen(reps)
    timing()
    sys.exit(1 if bad else 0)
