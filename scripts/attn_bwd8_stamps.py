"""Per-wave phase anatomy of the 8-wave attention backward (attn_bwd8) from the stamps build (diagnostic):

    make -C sparse-vae_amd stamps
    SVAE_LIB=sparse-vae_amd/sparse_vae/libsvae_stamps.so python scripts/attn_bwd8_stamps.py

For the first 1024 hardware blocks of one launch at the C2 decoder shape (B 64, H 8, L 512, hd 64, causal): cycle sums
per wave of the prologue, the S / dP / dV / dK phase (with the dS^T writes), the wait at the dS^T barrier, the dQ phase,
the end-of-tile wait + barrier and the epilogue, by key block class (q-tiles swept) and by wave.
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
N.lib.svae_debug_bwd8_stamps.argtypes = [ctypes.c_void_p]
PH = ['prologue', 'S/dP/dV/dK', 'dS barrier', 'dQ', 'end wait+barrier', 'epilogue']


def run(B, L, hd, causal=True):
    H = 8
    d = H * hd
    torch.manual_seed(0)
    qkv = torch.randn(B * L, 3 * d, device=dev).bfloat16()
    o = torch.empty(B * L, d, device=dev).bfloat16()
    o32 = torch.empty(B * L, d, device=dev)
    lse = torch.empty(B, H, L, device=dev)
    kw = dict(B=B, H=H, Lq=L, Lk=L, hd=hd, sq=3 * d, sk=3 * d, sv=3 * d, so=d, bq=L * 3 * d, bk=L * 3 * d,
              bv=L * 3 * d, bo=L * d, causal=causal, o32=o32, so32=d, bo32=L * d)
    K.attention(qkv, qkv[:, d:], qkv[:, 2 * d:], o, lse, **kw)
    dout = torch.randn(B * L, d, device=dev).bfloat16()
    dqkv = torch.empty(B * L, 3 * d, device=dev).bfloat16()
    delta = torch.empty(B, H, L, device=dev)
    part = torch.empty(K.attn_dq_part_elems(B, H, L, L, hd), device=dev)
    for _ in range(3):
        K.attention(qkv, qkv[:, d:], qkv[:, 2 * d:], o, lse, backward=True, dout=dout, sdo=d, bdo=L * d,
                    delta=delta, dq_bf=dqkv, ldq_bf=3 * d, dk=dqkv[:, d:], dv=dqkv[:, 2 * d:], sdk=3 * d,
                    sdv=3 * d, bdk=L * 3 * d, bdv=L * 3 * d, dq_part=part, **kw)
    torch.cuda.synchronize()
    buf = np.zeros((1024, 8, 8), dtype=np.uint64)
    assert N.lib.svae_debug_bwd8_stamps(buf.ctypes.data) == 0
    s = buf.astype(np.int64)
    nblk = min(1024, (L + 255) // 256 * H * B)
    s = s[:nblk]
    nq = s[:, 0, 7]
    print(f'B={B} L={L} hd={hd} causal={int(causal)}: {nblk} blocks; cycles per wave (median over blocks and waves)',
          flush=True)
    for c in sorted(set(nq.tolist())):
        sel = s[nq == c]
        tot = sel[:, :, :6].sum(axis=2)
        line = '  '.join(f'{PH[k]} {np.median(sel[:, :, k]):7.0f}' for k in range(6))
        print(f'  key blocks sweeping {c} q-tiles ({len(sel)} blocks): total {np.median(tot):7.0f}  {line}  '
              f'live q-tiles/wave {np.median(sel[:, :, 6]):.1f}', flush=True)
        for w in range(8):
            ww = sel[:, w]
            print(f'     wave {w}: ' + '  '.join(f'{np.median(ww[:, k]):7.0f}' for k in range(6)) +
                  f'   live {np.median(ww[:, 6]):.0f}', flush=True)


if __name__ == '__main__':
    run(64, 512, 64)
    run(64, 1024, 96)
