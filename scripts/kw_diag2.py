"""Which K-tile's weights a stale k-weight slot read returns (diagnostic build libsvae_kw1.so, DMA stagger on):
weights w_t = (t mod 8) + 1 on every column k of K-tile t, A in [-64, 64]. A wrong row whose error is
(w_t' - w_t) S_t(m) for exactly one (t, t' - t), |t' - t| <= 3, is counted under t' - t.

    SVAE_LIB=$PWD/sparse-vae_amd/sparse_vae/libsvae_kw1.so python scripts/kw_diag2.py
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
g = torch.Generator(device=dev).manual_seed(5)
Kk, M, Nn = 32768, 4096, 512
nt = Kk // 64
A = torch.randint(-64, 65, (Kk, M), device=dev, generator=g).float()
B = torch.randint(-2, 3, (Kk, Nn), device=dev, generator=g).float()
Ab, Bb = A.bfloat16(), B.bfloat16()
S = A.view(nt, 64, M).sum(1).cpu().long()
wt = torch.tensor([(t % 8) + 1 for t in range(nt)])
kw = wt.repeat_interleave(64).float().to(dev)
want = (S * wt[:, None]).sum(0)
C = torch.empty(M, Nn, device=dev)
hist = collections.Counter()
for rep in range(8):
    rs = torch.zeros(M, device=dev)
    K.gemm(Ab, Bb, C, M, Nn, Kk, a_t=True, b_t=True, ldb=Nn, epi=N.EPI_F32_ACC, a_rowsum=rs, k_weight=kw)
    torch.cuda.synchronize()
    got = rs.cpu().double().round().long()
    bad = (got != want).nonzero().flatten().tolist()
    for m in bad:
        err = int(got[m] - want[m])
        cands = []
        for t in range(nt):
            s = int(S[t][m])
            if s == 0 or err % s:
                continue
            q = err // s                      # = w_t' - w_t
            for dt in (-3, -2, -1, 1, 2, 3):
                t2 = t + dt
                if 0 <= t2 < nt and int(wt[t2] - wt[t]) == q:
                    cands.append((t, dt))
        rl = m % 256
        key = ('wr%d' % (rl // 128), 'wc%d' % ((rl % 128) // 32))
        if len(cands) == 1:
            hist[key + ('dt%+d' % cands[0][1], 'pos %s' % ('first' if cands[0][0] < 2 else 'last' if cands[0][0] >= nt - 2 else 'mid'))] += 1
        else:
            hist[key + ('ambiguous' if cands else 'unexplained',)] += 1
    print(f'rep {rep}: {len(bad)} wrong rows', flush=True)
print('classes:', dict(hist.most_common(30)))
