"""Which tiles / rows / K-tiles of an 8-phase gemm256 launch come out wrong (SVAE_GEMM8=1): integer operands, exact
reference; per 256 x 256 tile the count of wrong elements, and for the first wrong tile the error pattern."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'sparse-vae_amd'))
import torch  # noqa: E402
from sparse_vae import kernels as K  # noqa: E402
from sparse_vae import _native as N  # noqa: E402

dev = torch.device('cuda', 0)


def run(M, Nn, Kk, bt=False, reps=3):
    torch.manual_seed(M + Kk)
    Ai = torch.randint(-2, 3, (M, Kk), device=dev).float()
    Bi = torch.randint(-2, 3, (Nn, Kk), device=dev).float()
    ref = Ai @ Bi.t()
    Bs = Bi.t().contiguous() if bt else Bi
    for r in range(reps):
        C = torch.full((M, Nn), 12345.0, device=dev)
        K.gemm(Ai.bfloat16(), Bs.bfloat16(), C, M, Nn, Kk, b_t=bt, ldb=Nn if bt else Kk, epi=N.EPI_F32)
        torch.cuda.synchronize()
        bad = C != ref
        nb = int(bad.sum())
        print(f'M={M} N={Nn} K={Kk} bt={bt} rep {r}: {nb} wrong of {M * Nn}', flush=True)
        if nb:
            tm, tn = (M + 255) // 256, (Nn + 255) // 256
            tiles = []
            for i in range(tm):
                for j in range(tn):
                    c = int(bad[i * 256:(i + 1) * 256, j * 256:(j + 1) * 256].sum())
                    if c:
                        tiles.append((i, j, c))
            print('  wrong tiles (tm, tn, count):', tiles[:20], 'of', len(tiles), 'tiles; grid', tm, 'x', tn)
            i, j, _ = tiles[0]
            blk = bad[i * 256:(i + 1) * 256, j * 256:(j + 1) * 256]
            rows = blk.any(1).nonzero().flatten().tolist()
            cols = blk.any(0).nonzero().flatten().tolist()
            print('  first tile wrong rows', rows[:12], '...', len(rows), ' cols', cols[:12], '...', len(cols))
            d = (C - ref)[i * 256:(i + 1) * 256, j * 256:(j + 1) * 256][blk]
            print('  diff sample', d[:10].tolist(), 'C sample', C[i * 256:(i + 1) * 256, j * 256:(j + 1) * 256][blk][:5].tolist())


if __name__ == '__main__':
    run(8200, 2056, 520)
    run(8192, 2048, 512)
    run(8192, 2048, 520)
    run(8200, 2056, 512)
    run(2048, 2048, 4096)
