"""Per-tile cycle anatomy of gemm256 from the stamps build (diagnostic):

    make -C sparse-vae_amd stamps
    SVAE_LIB=sparse-vae_amd/sparse_vae/libsvae_stamps.so python scripts/gemm_stamps.py
For each case: median cycles per tile of the K loop and of the epilogue (blocks 0..7, tiles after the first).
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'sparse-vae_amd'))
import torch  # noqa: E402
from sparse_vae import kernels as K  # noqa: E402
from sparse_vae import _native as N  # noqa: E402

dev = torch.device('cuda', 0)
bf16 = torch.bfloat16
N.lib.svae_debug_stamps.argtypes = [ctypes.c_void_p]
N.lib.svae_debug_stamps_clear.argtypes = []


def stamps():
    buf = np.zeros((8, 96, 3), dtype=np.uint64)
    torch.cuda.synchronize()
    assert N.lib.svae_debug_stamps(buf.ctypes.data) == 0
    return buf.astype(np.int64)


def report(name, fn):
    zero = np.zeros((8, 96, 3), dtype=np.uint64)
    N.lib.svae_debug_stamps_clear()
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s = stamps()
    ntiles = int((s[0, :, 0] > 0).sum())
    loop = s[:, 1:ntiles, 1] - s[:, 1:ntiles, 0]
    epi = s[:, 1:ntiles, 2] - s[:, 1:ntiles, 1]
    gap = s[:, 2:ntiles, 0] - s[:, 1:ntiles - 1, 2]
    if ntiles == 1:   # one tile per block: the first (cold) tile is all there is
        loop, epi = s[:, :1, 1] - s[:, :1, 0], s[:, :1, 2] - s[:, :1, 1]
    print(f'{name:28s} tiles/block {ntiles:3d}  K-loop {np.median(loop):8.0f} cyc  epilogue {np.median(epi):7.0f} cyc  '
          f'between {np.median(gap) if gap.size else 0:6.0f} cyc', flush=True)


T, d, V = 32768, 512, 32768
h = torch.randn(T, d, device=dev).to(bf16)
W = (0.02 * torch.randn(V, d, device=dev)).to(bf16)
bias = torch.zeros(V, device=dev)
logits = torch.empty(T, V, dtype=bf16, device=dev)
part = torch.empty(T, V // 128, 2, device=dev)
labels = torch.randint(3, V, (T,), dtype=torch.int32, device=dev)
lab = torch.empty(T, device=dev)
report('head bf16', lambda: K.gemm(h, W, logits, T, V, d, epi=N.EPI_BF16, bias=bias))
report('head ce_stats', lambda: K.gemm(h, W, logits, T, V, d, epi=N.EPI_CE_STATS, bias=bias, aux=part,
                                       labels=labels, label_logit=lab))
row_a = torch.randn(T, device=dev)
report('head ce_prob', lambda: K.gemm(h, W, logits, T, V, d, epi=N.EPI_CE_PROB, bias=bias, aux=part, labels=labels,
                                      row_a=row_a))
W1 = (0.02 * torch.randn(2048, d, device=dev)).to(bf16)
f = torch.empty(T, 2048, dtype=bf16, device=dev)
gp = torch.empty(T, 2048, dtype=bf16, device=dev)
report('ffn1 bf16', lambda: K.gemm(h, W1, f, T, 2048, d, epi=N.EPI_BF16))
report('ffn1 gelu', lambda: K.gemm(h, W1, f, T, 2048, d, epi=N.EPI_GELU, bias=bias[:2048], aux=gp, ldaux=2048))
x32 = torch.randn(T, d, device=dev)
o32 = torch.empty(T, d, device=dev)
hb = torch.randn(T, 2048, device=dev).to(bf16)
W2 = (0.02 * torch.randn(d, 2048, device=dev)).to(bf16)
Wo = (0.02 * torch.randn(d, d, device=dev)).to(bf16)
report('outproj f32+resid', lambda: K.gemm(h, Wo, o32, T, d, d, epi=N.EPI_F32, bias=bias[:d], resid=x32, ldr=d))
report('outproj bf16', lambda: K.gemm(h, Wo, f[:, :d], T, d, d, epi=N.EPI_BF16, ldc=2048))
report('ffn2 bf16', lambda: K.gemm(hb, W2, f[:, :d], T, d, 2048, epi=N.EPI_BF16, ldc=2048))
report('ffn2 drop+resid', lambda: K.gemm(hb, W2, o32, T, d, 2048, epi=N.EPI_DROPOUT_RESID, resid=x32, ldr=d,
                                         drop_p=0.1, seed=3))
report('ffn2 resid (p=0)', lambda: K.gemm(hb, W2, o32, T, d, 2048, epi=N.EPI_DROPOUT_RESID, resid=x32, ldr=d,
                                          drop_p=0.0, seed=3))
report('ffn1-dX gelu_bwd', lambda: K.gemm(h, W1, f, T, 2048, d, epi=N.EPI_GELU_BWD, aux=gp, ldaux=2048))
A8 = torch.randn(8192, 8192, device=dev).to(bf16)
C8 = torch.empty(8192, 8192, device=dev, dtype=bf16)
report('8K^3 bf16', lambda: K.gemm(A8, A8, C8, 8192, 8192, 8192, epi=N.EPI_BF16))

# split-K weight-gradient pairs (one tile per block: the K loop covers the block's whole K slice) and the clock the
# stamps count at (s_memtime cycles of block 0's tile against HIP-event time of the same launch)
dY2 = torch.randn(T, 2048, device=dev).to(bf16)
Wg1 = torch.zeros(2048, d, device=dev)
Wg2 = torch.zeros(d, 2048, device=dev)
ffn_pair = lambda: K.linear_dw_pair((dY2, h, Wg1, T, 2048, d, None, None, None),   # noqa: E731
                                    (h, dY2, Wg2, T, d, 2048, None, None, None))
report('ffn dW pair (64 K-tiles)', ffn_pair)
dq = torch.randn(T, 1536, device=dev).to(bf16)
Wq = torch.zeros(1536, d, device=dev)
Wo2 = torch.zeros(d, d, device=dev)
bq, bo = torch.zeros(1536, device=dev), torch.zeros(d, device=dev)
qkv_pair = lambda: K.linear_dw_pair((dq, h, Wq, T, 1536, d, None, None, bq),   # noqa: E731
                                    (h, h, Wo2, T, d, d, None, None, bo))
report('qkv+out dW pair (32 K-tiles)', qkv_pair)
# the transposed K-step alone: 8K^3 dY^T X layout, one FFN1 dW tile column without splits (16 blocks: no contention),
# and the same GEMM split 16 ways (256 blocks)
C8f = torch.zeros(8192, 8192, device=dev)
report('8K^3 at bt f32_acc', lambda: K.gemm(A8, A8, C8f, 8192, 8192, 8192, a_t=True, b_t=True, epi=N.EPI_F32_ACC))
dY4, h4 = dY2[:4096], h[:4096]
report('ffn1 dW K=4096 16 blocks', lambda: K.gemm(dY4, h4, Wg1, 2048, d, 4096, a_t=True, b_t=True, lda=2048, ldb=d,
                                                    ldc=d, epi=N.EPI_F32_ACC))
report('ffn1 dW K=32768 split 16', lambda: K.linear_dw(dY2, h, Wg1, T, 2048, d))
h8 = torch.randn(4096, 8192, device=dev).to(bf16)
report('8K^2 x K=4096 at bt (256 blk)', lambda: K.gemm(h8, h8, C8f, 8192, 8192, 4096, a_t=True, b_t=True,
                                                        epi=N.EPI_F32_ACC))
for name, fn in (('ffn dW pair', ffn_pair), ('qkv+out dW pair', qkv_pair), ('8K^3', lambda: K.gemm(
        A8, A8, C8, 8192, 8192, 8192, epi=N.EPI_BF16))):
    N.lib.svae_debug_stamps_clear()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    N.lib.svae_debug_stamps_clear()
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    s = stamps()
    nt = int((s[0, :, 0] > 0).sum())
    span = int(s[:, nt - 1, 2].max() - s[:, 0, 0].min())
    us = e0.elapsed_time(e1) * 1e3
    print(f'{name:28s} launch {us:8.1f} us  blocks 0-7 span {span} cyc -> {span / us:7.0f} MHz lower bound', flush=True)
