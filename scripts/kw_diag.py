"""Classify the k-weighted row-sum failures of an LDS-slot diagnostic build (SVAE_LIB=.../libsvae_kw1.so). The
weights are 1 on the K-tiles t = 0 (mod 4) and 0 elsewhere, so the two LDS stages alternate between a tile with ones
and one with zeros every other K-tile. A wrong row's error is matched against a single K-tile sum S_t(m) (A in
[-64, 64], so the sums rarely collide): -S_t with t = 0 (mod 4): tile t's weights read as zeros (stale or early);
+S_t with t = 2 (mod 4): tile t's zero weights read as the ones of a tile two away. Reported with the K-tile position
and the wave (wave row wr, column wave wc) that computed the row.

    SVAE_LIB=$PWD/sparse-vae_amd/sparse_vae/libsvae_kw1.so python scripts/kw_diag.py
"""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'sparse-vae_amd'))
import torch  # noqa: E402
from sparse_vae import kernels as K  # noqa: E402
from sparse_vae import _native as N  # noqa: E402

dev = torch.device('cuda', 0)
g = torch.Generator(device=dev).manual_seed(3)
total = collections.Counter()
for Kk, M, Nn in ((32768, 4096, 512), (2048, 16384, 776)):
    A = torch.randint(-64, 65, (Kk, M), device=dev, generator=g).float()
    B = torch.randint(-2, 3, (Kk, Nn), device=dev, generator=g).float()
    Ab, Bb = A.bfloat16(), B.bfloat16()
    nt = Kk // 64
    S = A.view(nt, 64, M).sum(1).cpu()            # S[t][m]: the K-tile sums
    kw = torch.zeros(Kk, device=dev)
    for t in range(0, nt, 4):
        kw[64 * t:64 * t + 64] = 1.0
    want = S[0::4].sum(0)
    C = torch.empty(M, Nn, device=dev)
    for rep in range(6):
        rs = torch.zeros(M, device=dev)
        C.zero_()
        K.gemm(Ab, Bb, C, M, Nn, Kk, a_t=True, b_t=True, ldb=Nn, epi=N.EPI_F32_ACC, a_rowsum=rs, k_weight=kw)
        torch.cuda.synchronize()
        rs = rs.cpu()
        bad = (rs != want).nonzero().flatten().tolist()
        cls = collections.Counter()
        for m in bad:
            err = rs[m].item() - want[m].item()
            lost = [t for t in range(0, nt, 4) if S[t][m].item() == -err]
            gained = [t for t in range(2, nt, 4) if S[t][m].item() == err]
            rl = m % 256
            wr, wc = rl // 128, (rl % 128) // 32
            if len(lost) + len(gained) == 1:
                kind, t = ('lost', lost[0]) if lost else ('gained', gained[0])
                pos = 'first' if t < 2 else ('last' if t >= nt - 2 else 'mid')
                cls[(kind, pos, f'wr{wr}', f'wc{wc}')] += 1
            else:
                cls[('ambiguous' if lost or gained else 'other', f'wr{wr}', f'wc{wc}')] += 1
        total.update(cls)
        print(f'K={Kk} M={M} N={Nn} rep {rep}: {len(bad):4d} wrong rows', dict(cls.most_common(8)), flush=True)
print('total by class:', dict(total.most_common(30)))
