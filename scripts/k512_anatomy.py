"""Anatomy of the one-tile-per-CU K = 512 GEMMs from the stamps build:

    make -C sparse-vae_amd stamps
    SVAE_LIB=sparse-vae_amd/sparse_vae/libsvae_stamps.so python scripts/k512_anatomy.py

Per case: HIP-event time of one launch; for blocks 0..7 (one per XCD) the s_memtime cycles from the earliest block's
first stamp to each block's tile start, K-loop end and epilogue end (max over the 8 blocks), converted to us with the
clock measured on the 8K^3 launch (span of the stamps / event time).
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
N.lib.svae_debug_rt.argtypes = [ctypes.c_void_p]


def realtime(nblk):
    rt = np.zeros((1024, 2), dtype=np.uint64)
    assert N.lib.svae_debug_rt(rt.ctypes.data) == 0
    rt = rt[:nblk].astype(np.int64)
    t0 = rt[:, 0].min()
    st, en = (rt[:, 0] - t0) / 100.0, (rt[:, 1] - t0) / 100.0      # 100 MHz -> us
    return (f'entry skew p50 {np.median(st):4.1f} p90 {np.percentile(st, 90):4.1f} max {st.max():4.1f} us, '
            f'exit p10 {np.percentile(en, 10):5.1f} p50 {np.median(en):5.1f} max {en.max():5.1f} us')


def run(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    N.lib.svae_debug_stamps_clear()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    buf = np.zeros((8, 96, 3), dtype=np.uint64)
    assert N.lib.svae_debug_stamps(buf.ctypes.data) == 0
    return buf.astype(np.int64), e0.elapsed_time(e1) * 1e3


T, d = 32768, 512
h = torch.randn(T, d, device=dev).to(bf16)
hb = torch.randn(T, 2048, device=dev).to(bf16)
A8 = torch.randn(8192, 8192, device=dev).to(bf16)
C8 = torch.empty(8192, 8192, device=dev, dtype=bf16)
s, us = run(lambda: K.gemm(A8, A8, C8, 8192, 8192, 8192, epi=N.EPI_BF16))
nt = int((s[0, :, 0] > 0).sum())
print('raw 8K^3 block stamps (tile 0):', s[:, 0, :].tolist(), 'tiles', nt, flush=True)
mhz = float(np.median(s[:, nt - 1, 2] - s[:, 0, 0])) / us   # per-XCD clocks: spans within a block only
print(f'clock from 8K^3: {mhz:.0f} cycles per us (event {us:.1f} us)', flush=True)

Wo = (0.02 * torch.randn(d, d, device=dev)).to(bf16)
W1 = (0.02 * torch.randn(2048, d, device=dev)).to(bf16)
W2 = (0.02 * torch.randn(d, 2048, device=dev)).to(bf16)
bias = torch.zeros(2048, device=dev)
x32 = torch.randn(T, d, device=dev)
o32 = torch.empty(T, d, device=dev)
ob = torch.empty(T, d, device=dev, dtype=bf16)
f = torch.empty(T, 2048, dtype=bf16, device=dev)
gp = torch.empty(T, 2048, dtype=bf16, device=dev)
cases = [
    ('K512 f32', lambda: K.gemm(h, Wo, o32, T, d, d, epi=N.EPI_F32)),
    ('K512 f32+resid', lambda: K.gemm(h, Wo, o32, T, d, d, epi=N.EPI_F32, bias=bias[:d], resid=x32, ldr=d)),
    ('K512 bf16', lambda: K.gemm(h, Wo, ob, T, d, d, epi=N.EPI_BF16)),
    ('K64 bf16 (no K-loop)', lambda: K.gemm(h[:, :64], Wo[:, :64], ob, T, d, 64, lda=d, ldb=d, epi=N.EPI_BF16)),
    ('K2048 drop+resid', lambda: K.gemm(hb, W2, o32, T, d, 2048, epi=N.EPI_DROPOUT_RESID, resid=x32, ldr=d,
                                        drop_p=0.1, seed=3)),
    ('ffn1 gelu (4 tiles)', lambda: K.gemm(h, W1, f, T, 2048, d, epi=N.EPI_GELU, bias=bias, aux=gp, ldaux=2048)),
    ('ffn1 bf16 (4 tiles)', lambda: K.gemm(h, W1, f, T, 2048, d, epi=N.EPI_BF16)),
]
for name, fn in (('memset 32 MB', lambda: ob.zero_()), ('memset 64 MB', lambda: o32.zero_()),
                 ('copy 32 MB', lambda: ob.copy_(h))):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        fn()
    e1.record()
    torch.cuda.synchronize()
    print(f'{name:22s} event {e0.elapsed_time(e1) * 100:6.1f} us', flush=True)
for name, fn in cases:
    s, us = run(fn)
    nt = int((s[0, :, 0] > 0).sum())
    ok = (s[:, 0, 0] > 0)
    rows = []
    for t in range(nt):
        kl = np.median(s[ok, t, 1] - s[ok, t, 0]) / mhz
        ep = np.median(s[ok, t, 2] - s[ok, t, 1]) / mhz
        gap = np.median(s[ok, t, 0] - s[ok, t - 1, 2]) / mhz if t else 0.0
        rows.append(f't{t}: gap {gap:4.1f} kloop {kl:5.1f} epi {ep:5.1f}')
    tot = np.median(s[ok, nt - 1, 2] - s[ok, 0, 0]) / mhz
    print(f'{name:22s} event {us:6.1f} us | stamped {tot:5.1f} us | ' + ' | '.join(rows), flush=True)
    print(f'{"":22s} 256 blocks: ' + realtime(256), flush=True)
