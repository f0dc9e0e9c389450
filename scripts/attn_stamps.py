"""Per-block cycle anatomy of the attention forward from the stamps build (diagnostic):

    make -C sparse-vae_amd stamps
    SVAE_LIB=sparse-vae_amd/sparse_vae/libsvae_stamps.so python scripts/attn_stamps.py
For the first 1024 hardware blocks of one launch at the C2 decoder shape: start-time spread, prologue (block start to
the first K/V tile's barrier: Q fragments + first DMA), key loop per visited tile, epilogue (O, o32, lse stores).
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
N.lib.svae_debug_attn_stamps.argtypes = [ctypes.c_void_p]


def run(B, L, causal, with_o32=True):
    H, hd = 8, 64
    d = H * hd
    qkv = torch.randn(B * L, 3 * d, device=dev).bfloat16()
    o = torch.empty(B * L, d, device=dev).bfloat16()
    o32 = torch.empty(B * L, d, device=dev)
    lse = torch.empty(B, H, L, device=dev)
    kw = dict(B=B, H=H, Lq=L, Lk=L, hd=hd, sq=3 * d, sk=3 * d, sv=3 * d, so=d, bq=L * 3 * d, bk=L * 3 * d,
              bv=L * 3 * d, bo=L * d, causal=causal, o32=o32 if with_o32 else None, so32=d, bo32=L * d)
    for _ in range(3):
        K.attention(qkv, qkv[:, d:], qkv[:, 2 * d:], o, lse, **kw)
    torch.cuda.synchronize()
    buf = np.zeros((1024, 6), dtype=np.uint64)
    assert N.lib.svae_debug_attn_stamps(buf.ctypes.data) == 0
    s = buf.astype(np.int64)
    t0 = s[:, 0].min()
    start, first, loop_end, end, nv, qt = (s[:, i] for i in range(6))
    pro = first - start
    per_tile = (loop_end - first) / np.maximum(nv, 1)
    epi = end - loop_end
    total = end - start
    print(f'B={B} L={L} causal={int(causal)} o32={int(with_o32)}: blocks 0..1023 start spread '
          f'{np.percentile(start - t0, 50):.0f}/{np.percentile(start - t0, 90):.0f}/{(start - t0).max():.0f} cyc '
          f'(p50/p90/max); per block: total {np.median(total):.0f}, prologue {np.median(pro):.0f}, '
          f'loop {np.median(loop_end - first):.0f} = {np.median(per_tile):.0f}/tile x {np.median(nv):.0f}, '
          f'epilogue {np.median(epi):.0f} cyc', flush=True)
    for q in range(int(qt.max()) + 1):
        sel = qt == q
        if sel.any():
            print(f'   q-tile {q}: tiles {np.median(nv[sel]):.0f}  total {np.median(total[sel]):.0f}  prologue '
                  f'{np.median(pro[sel]):.0f}  per tile {np.median(per_tile[sel]):.0f}  epilogue {np.median(epi[sel]):.0f}',
                  flush=True)


if __name__ == '__main__':
    run(64, 512, True)
    run(64, 512, False)
    run(64, 512, True, with_o32=False)
