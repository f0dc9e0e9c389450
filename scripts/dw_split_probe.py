"""Split-K choices for the step's weight-gradient GEMMs (dW[n_out, n_in] += dY^T X over T = 32768 rows), timed with
the slab reduction: python scripts/dw_split_probe.py"""
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
    return e0.elapsed_time(e1) / reps * 1e3


T = 32768
RS = os.environ.get('DW_RS') == '1'   # with the fused bias-gradient row sums (as in the step)
for n_out, n_in in [(512, 512), (1024, 512), (1536, 512), (2048, 512), (512, 2048)]:
    dY = torch.randn(T, n_out, device=dev).bfloat16()
    X = torch.randn(T, n_in, device=dev).bfloat16()
    Wg = torch.zeros(n_out, n_in, device=dev)
    bg = torch.zeros(n_out, device=dev) if RS else None
    auto = K.auto_splits(n_out, n_in, T)
    for s in sorted({auto, 16, 32, 64, 128}):
        if T // s < 256:
            continue
        slab = K._slab_workspace(s * n_out * n_in, dev) if s > 1 else None

        def fn():
            K.gemm(dY, X, Wg, n_out, n_in, T, a_t=True, b_t=True, lda=n_out, ldb=n_in, ldc=n_in,
                   epi=N.EPI_F32_ATOMIC if s > 1 else N.EPI_F32_ACC, splits=s, aux=slab, a_rowsum=bg)
        us = timeit(fn)
        print(f'dW{" rs" if RS else ""} impl={os.environ.get("SVAE_GEMM_IMPL", "0")} {n_out}x{n_in} K={T} splits={s:4d}{" (auto)" if s == auto else "       "} {us:8.1f} us '
              f'{2.0 * n_out * n_in * T / us / 1e6:7.1f} TF/s', flush=True)
