"""Time the LayerNorm forward alone at the C4 / C5 row shape (65,536 rows x 768, f32 in, bf16 out: 6 B per element)
and its z-splice form; variants through SVAE_LN_FWD_4COL / SVAE_LN_FWD_BLOCKS.

    python scripts/ln_probe.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'sparse-vae_amd'))
import torch  # noqa: E402
from sparse_vae import kernels as K  # noqa: E402

dev = torch.device('cuda', 0)


def timeit(fn, reps=30):
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
    for rows, D in ((65536, 768), (32768, 512)):
        x = torch.randn(rows, D, device=dev)
        w, b = torch.randn(D, device=dev), torch.randn(D, device=dev)
        y = torch.empty(rows, D, device=dev, dtype=torch.bfloat16)
        mean, rstd = torch.empty(rows, device=dev), torch.empty(rows, device=dev)
        zrows = torch.randn(rows // 1024, D, device=dev)
        t = timeit(lambda: K.layernorm_fwd(x, w, b, y, mean, rstd, rows, D))
        tz = timeit(lambda: K.layernorm_fwd_z(x, zrows, 1024, w, b, y, mean, rstd, rows, D))
        ref = torch.nn.functional.layer_norm(x, (D,), w, b)
        K.layernorm_fwd(x, w, b, y, mean, rstd, rows, D)
        err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
        gb = rows * D * 6 / 1e9
        print(f'rows={rows} D={D}  fwd {t:7.1f} us {gb / t * 1e6:7.1f} GB/s   fwd_z {tz:7.1f} us   max rel err {err:.2e}',
              flush=True)


if __name__ == '__main__':
    main()
