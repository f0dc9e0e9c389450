"""Calibration: libsvae GEMMs vs the vendor library (torch.matmul -> hipBLASLt) on the C2 step's shapes.

    python scripts/gemm_vs_blas.py
One line per shape: libsvae plain-epilogue time, hipBLASLt time, TF/s of each. Measurement only: the product
path never calls hipBLASLt (the fused epilogues are the point of the hand-written kernels).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'sparse-vae_amd'))
import torch  # noqa: E402
from sparse_vae import kernels as K  # noqa: E402
from sparse_vae import _native as N  # noqa: E402

dev = torch.device('cuda', 0)
bf16 = torch.bfloat16


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
    shapes = [  # (M, N, K, tag): forward layout C = A . W^T
        (32768, 32768, 512, 'head fwd'),
        (32768, 2048, 512, 'FFN1 fwd'),
        (32768, 1536, 512, 'QKV fwd'),
        (32768, 512, 2048, 'FFN2 fwd'),
        (32768, 512, 512, 'out-proj fwd'),
        (32768, 512, 32768, 'head dX'),
        (8192, 8192, 8192, 'square 8K'),
    ]
    for M, N_, K_, tag in shapes:
        A = torch.randn(M, K_, device=dev).to(bf16)
        W = torch.randn(N_, K_, device=dev).to(bf16)
        C = torch.empty(M, N_, device=dev, dtype=bf16)
        fl = 2.0 * M * N_ * K_
        t_svae = timeit(lambda: K.gemm(A, W, C, M, N_, K_, epi=N.EPI_BF16))
        Wt = W.t()
        t_blas = timeit(lambda: torch.matmul(A, Wt, out=C))
        print(f'{tag:13s} M={M:6d} N={N_:6d} K={K_:6d}  libsvae {t_svae * 1e3:8.1f} us {fl / t_svae / 1e9:7.1f} TF/s   '
              f'hipBLASLt {t_blas * 1e3:8.1f} us {fl / t_blas / 1e9:7.1f} TF/s', flush=True)
    # dW layout (C = dY^T . X, K = tokens)
    for M, N_, K_, tag in [(2048, 512, 32768, 'FFN1 dW'), (512, 512, 32768, 'out dW'), (32768, 512, 32768, 'head dW')]:
        dY = torch.randn(K_, M, device=dev).to(bf16)
        X = torch.randn(K_, N_, device=dev).to(bf16)
        C = torch.zeros(M, N_, device=dev)
        fl = 2.0 * M * N_ * K_
        t_svae = timeit(lambda: K.linear_dw(dY, X, C, K_, M, N_))
        t_blas = timeit(lambda: torch.matmul(dY.t(), X))
        print(f'{tag:13s} M={M:6d} N={N_:6d} K={K_:6d}  libsvae {t_svae * 1e3:8.1f} us {fl / t_svae / 1e9:7.1f} TF/s   '
              f'hipBLASLt {t_blas * 1e3:8.1f} us {fl / t_blas / 1e9:7.1f} TF/s', flush=True)


if __name__ == '__main__':
    main()
