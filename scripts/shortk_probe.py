"""Time the C2 step's short-K, epilogue-heavy GEMM shapes in isolation under the kernel the library picks (run with
SVAE_GEMM_IMPL=1|2|3 to force the 128-tile register-staged, the 128-tile LDS-DMA or the 256-tile persistent kernel):
the out-projection with its f32 residual (one 256 x 256 tile per CU), bf16 out, FFN1 GELU, FFN2 dropout + residual,
QKV rotary. HIP events, 30 reps.      SVAE_GEMM_IMPL=2 python scripts/shortk_probe.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'sparse-vae_amd'))
import torch  # noqa: E402
from sparse_vae import kernels as K  # noqa: E402
from sparse_vae import _native as N  # noqa: E402

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
    T, d = int(os.environ.get('SHORTK_T', 32768)), 512   # SHORTK_T=4096: the encoder's latent rows (B x 64)
    torch.manual_seed(0)
    impl = os.environ.get('SVAE_GEMM_IMPL', 'auto')
    x = torch.randn(T, d, device=dev).bfloat16()
    f = torch.randn(T, 4 * d, device=dev).bfloat16()
    w = (torch.randn(d, d, device=dev) * 0.05).bfloat16()
    w1 = (torch.randn(4 * d, d, device=dev) * 0.05).bfloat16()
    w2 = (torch.randn(d, 4 * d, device=dev) * 0.05).bfloat16()
    wq = (torch.randn(3 * d, d, device=dev) * 0.05).bfloat16()
    b, b1, bq = torch.randn(d, device=dev), torch.randn(4 * d, device=dev), torch.randn(3 * d, device=dev)
    resid = torch.randn(T, d, device=dev)
    out32 = torch.empty(T, d, device=dev)
    out16 = torch.empty(T, d, device=dev, dtype=torch.bfloat16)
    h1 = torch.empty(T, 4 * d, device=dev, dtype=torch.bfloat16)
    gp = torch.empty(T, 4 * d, device=dev, dtype=torch.bfloat16)
    qkv = torch.empty(T, 3 * d, device=dev, dtype=torch.bfloat16)
    rot = torch.randn(T, d, device=dev)   # (cos, sin) pairs: any values time the same
    cases = [
        ('out-proj f32 + resid  N 512 K 512', 2 * T * d * d,
         lambda: K.gemm(x, w, out32, T, d, d, epi=N.EPI_F32, bias=b, resid=resid, ldr=d)),
        ('bf16 out              N 512 K 512', 2 * T * d * d, lambda: K.gemm(x, w, out16, T, d, d, epi=N.EPI_BF16)),
        ('FFN1 GELU             N 2048 K 512', 2 * T * 4 * d * d,
         lambda: K.gemm(x, w1, h1, T, 4 * d, d, epi=N.EPI_GELU, bias=b1, aux=gp, ldaux=4 * d)),
        ('FFN2 dropout + resid  N 512 K 2048', 2 * T * 4 * d * d,
         lambda: K.gemm(f, w2, out32, T, d, 4 * d, epi=N.EPI_DROPOUT_RESID, resid=resid, ldr=d, drop_p=0.1, seed=7)),
        ('QKV rotary            N 1536 K 512', 2 * T * 3 * d * d,
         lambda: K.gemm(x, wq, qkv, T, 3 * d, d, epi=N.EPI_ROTARY_BF16, bias=bq, rot=rot, rot_cols=2 * d, rot_d=d,
                        rot_seq=min(T, 512))),
    ]
    for name, flop, fn in cases:
        t = timeit(fn)
        print(f'impl {impl}: {name}: {t:7.1f} us  {flop / t / 1e6:7.1f} TF/s', flush=True)


if __name__ == '__main__':
    main()
