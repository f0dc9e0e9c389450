"""Time the vocabulary-head GEMM variants of the training step at the C2 shape (T = V = 32768, d = 512):
forward CE_STATS (logits) vs CE_PROB (P-head), dW with plain / weighted / no bias row sums, dX plain vs
ROWSCALE_GATHER.

    python scripts/head_probe.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'sparse-vae_amd'))
import torch  # noqa: E402
from sparse_vae import kernels as K  # noqa: E402
from sparse_vae import _native as N  # noqa: E402

dev = torch.device('cuda', 0)
bf16, f32 = torch.bfloat16, torch.float32


def timeit(fn, reps=10):
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
    T, d, V = 32768, 512, 32768
    torch.manual_seed(0)
    hh = torch.randn(T, d, device=dev).to(bf16)
    W = (0.05 * torch.randn(V, d, device=dev)).to(bf16)
    WT = W.t().contiguous()
    bias = torch.zeros(V, device=dev)
    labels = torch.randint(3, V, (T,), dtype=torch.int32, device=dev)
    out = torch.empty(T, V, dtype=bf16, device=dev)
    part2 = torch.empty(T, V // 128, 2, device=dev)
    part1 = torch.empty(V // 128, T, device=dev)
    ll = torch.empty(T, device=dev)
    coff = torch.empty(T, device=dev)
    K.ce_label_logit(hh, W, bias, labels, T, d, coff)
    dW = torch.zeros(V, d, device=dev)
    db = torch.zeros(V, device=dev)
    r = torch.rand(T, device=dev) * 1e-4
    q = torch.rand(T, device=dev) * 1e-4
    dhh = torch.empty(T, d, dtype=bf16, device=dev)
    hhT = hh.t().contiguous()
    fl = 2.0 * T * d * V
    cases = {
        'fwd CE_STATS': lambda: K.gemm(hh, W, out, T, V, d, epi=N.EPI_CE_STATS, bias=bias, aux=part2, labels=labels,
                                       label_logit=ll),
        'fwd CE_PROB': lambda: K.gemm(hh, W, out, T, V, d, epi=N.EPI_CE_PROB, bias=bias, aux=part1, labels=labels,
                                      row_a=coff),
        'fwd BF16': lambda: K.gemm(hh, W, out, T, V, d, epi=N.EPI_BF16, bias=bias),
        'dW no rowsum': lambda: K.gemm(out, hh, dW, V, d, T, a_t=True, b_t=True, lda=V, ldb=d, ldc=d,
                                       epi=N.EPI_F32_ACC),
        'dW rowsum': lambda: K.gemm(out, hh, dW, V, d, T, a_t=True, b_t=True, lda=V, ldb=d, ldc=d,
                                    epi=N.EPI_F32_ACC, a_rowsum=db),
        'dW rowsum kw': lambda: K.gemm(out, hh, dW, V, d, T, a_t=True, b_t=True, lda=V, ldb=d, ldc=d,
                                       epi=N.EPI_F32_ACC, a_rowsum=db, k_weight=r),
        'dW kw, B K-contig': lambda: K.gemm(out, hhT, dW, V, d, T, a_t=True, b_t=False, lda=V, ldb=T, ldc=d,
                                            epi=N.EPI_F32_ACC, a_rowsum=db, k_weight=r),
        'dW, B K-contig': lambda: K.gemm(out, hhT, dW, V, d, T, a_t=True, b_t=False, lda=V, ldb=T, ldc=d,
                                         epi=N.EPI_F32_ACC),
        'dX BF16': lambda: K.gemm(out, WT, dhh, T, d, V, epi=N.EPI_BF16),
        'dX ROWSCALE_GATHER': lambda: K.gemm(out, WT, dhh, T, d, V, epi=N.EPI_ROWSCALE_GATHER, labels=labels,
                                             row_a=r, row_b=q, gather=W, ldg=d),
    }
    for name, fn in cases.items():
        us = timeit(fn)
        print(f'{name:20s} {us:9.1f} us  {fl / us / 1e6:7.1f} TF/s', flush=True)


if __name__ == '__main__':
    main()
