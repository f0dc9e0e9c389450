"""Isolate the cost of the weight-gradient GEMM's operand layout (verdict r05 item 2): the same C = A^T B product at the
C2 dW shapes (split-K slabs, >= 192 blocks so the library takes gemm256 for both layouts) run as
  * TN  -- the product form: A = dY [K][M], B = X [K][N] (token-major), gemm256<1,1,SLAB> (transposed LDS reads);
  * TN+bias -- the same with the fused bias-gradient row sums (the QKV / FFN1 dW);
  * NT  -- the same numbers with K-contiguous copies A^T [M][K], B^T [N][K], gemm256<0,0,F32> in slab mode (row reads);
and the paired launches of the step (linear_dw_pair). Times by HIP events, 20 reps.   python scripts/tn_probe.py
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
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    for M, N_, T, splits in [(2048, 512, 32768, 16), (512, 2048, 32768, 16), (1536, 512, 32768, 16), (512, 512, 32768, 64)]:
        torch.manual_seed(0)
        dY = torch.randn(T, M, device=dev).bfloat16()
        X = torch.randn(T, N_, device=dev).bfloat16()
        dYt, Xt = dY.t().contiguous(), X.t().contiguous()
        slab = torch.empty(splits * M * N_, device=dev)
        C1, C2 = torch.zeros(M, N_, device=dev), torch.zeros(M, N_, device=dev)
        bg = torch.zeros(M, device=dev)
        flop = 2.0 * M * N_ * T

        def tn(bias=None):
            C1.zero_()
            K.gemm(dY, X, C1, M, N_, T, a_t=True, b_t=True, lda=M, ldb=N_, ldc=N_, epi=N.EPI_F32_ATOMIC, splits=splits,
                   a_rowsum=bias, aux=slab)

        def nt():
            C2.zero_()
            K.gemm(dYt, Xt, C2, M, N_, T, a_t=False, b_t=False, lda=T, ldb=T, ldc=N_, epi=N.EPI_F32_ATOMIC, splits=splits,
                   aux=slab)

        tn()
        nt()
        torch.cuda.synchronize()
        err = ((C1 - C2).abs().max() / C2.abs().max()).item()
        t_tn, t_tnb, t_nt = timeit(tn), timeit(lambda: tn(bg)), timeit(nt)
        z = torch.zeros(M, N_, device=dev)
        t_zero = timeit(lambda: z.zero_())
        print(f'M={M} N={N_} K={T} splits={splits}: TN {t_tn - t_zero:7.1f} us ({flop / (t_tn - t_zero) / 1e6:6.1f} TF/s)  '
              f'TN+bias {t_tnb - t_zero:7.1f} us  NT {t_nt - t_zero:7.1f} us ({flop / (t_nt - t_zero) / 1e6:6.1f} TF/s)  '
              f'(incl. slab reduce; C zero {t_zero:.1f} us subtracted)  TN vs NT max rel diff {err:.1e}', flush=True)


    T, d = 32768, 512
    h = torch.randn(T, d, device=dev).bfloat16()
    dY2 = torch.randn(T, 2048, device=dev).bfloat16()
    dq = torch.randn(T, 1536, device=dev).bfloat16()
    Wg1, Wg2 = torch.zeros(2048, d, device=dev), torch.zeros(d, 2048, device=dev)
    Wq, Wo = torch.zeros(1536, d, device=dev), torch.zeros(d, d, device=dev)
    b1, b2, bq, bo = (torch.zeros(n, device=dev) for n in (2048, d, 1536, d))
    for bias in (False, True):
        t = timeit(lambda: K.linear_dw_pair((dY2, h, Wg1, T, 2048, d, None, None, b1 if bias else None),
                                            (h, dY2, Wg2, T, d, 2048, None, None, b2 if bias else None)))
        print(f'pair ffn1+ffn2 dW (bias sums {bias}) {t:7.1f} us {2.0 * 2 * 2048 * d * T / t / 1e6:7.1f} TF/s', flush=True)
        t = timeit(lambda: K.linear_dw_pair((dq, h, Wq, T, 1536, d, None, None, bq if bias else None),
                                            (h, h, Wo, T, d, d, None, None, bo if bias else None)))
        print(f'pair qkv+out dW (bias sums {bias}) {t:7.1f} us {2.0 * (1536 + 512) * d * T / t / 1e6:7.1f} TF/s',
              flush=True)


if __name__ == '__main__':
    main()
