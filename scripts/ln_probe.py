"""Time the LayerNorm forward alone at the C4 / C5 row shape (65,536 rows x 768, f32 in, bf16 out: 6 B per element)
and its z-splice form; variants through SVAE_LN_FWD_4COL / SVAE_LN_FWD_BLOCKS. Then the decoder layers' backward at the
same shapes (dy bf16, x / dres f32 in, dx f32 + bf16 out: 16 B per element) against torch's LayerNorm backward.

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
        # the decoder layers' backward: dy bf16, x f32, dres f32 in; dx f32 + its bf16 copy out (16 B per element)
        dy = torch.randn(rows, D, device=dev).bfloat16()
        dres, dx = torch.randn(rows, D, device=dev), torch.empty(rows, D, device=dev)
        dx_bf = torch.empty(rows, D, device=dev, dtype=torch.bfloat16)
        wg = torch.zeros(2 * D, device=dev)
        part = torch.empty(1024 * 2 * D, device=dev)
        tb = timeit(lambda: K.layernorm_bwd(dy, x, w, mean, rstd, dres, dx, dx_bf, wg, rows, D, part))
        xt = x.clone().requires_grad_(True)
        torch.nn.functional.layer_norm(xt, (D,), w, None).backward(dy.float())
        K.layernorm_bwd(dy, x, w, mean, rstd, dres, dx, dx_bf, wg, rows, D, part)
        ref = xt.grad + dres
        errb = ((dx - ref).abs().max() / ref.abs().max()).item()
        gbb = rows * D * 16 / 1e9
        print(f'rows={rows} D={D}  bwd {tb:7.1f} us {gbb / tb * 1e6:7.1f} GB/s   max rel err {errb:.2e}', flush=True)


if __name__ == '__main__':
    main()
