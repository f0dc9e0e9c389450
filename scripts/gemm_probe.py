"""Time single GEMM launches of libsvae on the GPU (shape / epilogue experiments).

    python scripts/gemm_probe.py [head|all]
Prints one line per case: shape, epilogue, average launch time over 10 launches, TF/s.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'sparse-vae_amd'))
import torch  # noqa: E402
from sparse_vae import kernels as K  # noqa: E402
from sparse_vae import _native as N  # noqa: E402

dev = torch.device('cuda', 0)
bf16, f32 = torch.bfloat16, torch.float32


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def head_cases():
    T, d, V = 32768, 512, 32768
    h = torch.randn(T, d, device=dev).to(bf16)
    W = (0.02 * torch.randn(V, d, device=dev)).to(bf16)
    bias = torch.zeros(V, device=dev)
    logits = torch.empty(T, V, dtype=bf16, device=dev)
    part = torch.empty(T, V // 128, 2, device=dev)
    labels = torch.randint(3, V, (T,), dtype=torch.int32, device=dev)
    lab = torch.empty(T, device=dev)
    fl = 2.0 * T * d * V
    cases = {
        'bf16': lambda: K.gemm(h, W, logits, T, V, d, epi=N.EPI_BF16, bias=bias),
        'ce_stats': lambda: K.gemm(h, W, logits, T, V, d, epi=N.EPI_CE_STATS, bias=bias, aux=part, labels=labels,
                                   label_logit=lab),
        'ce_noC': lambda: K.gemm(h, W, None, T, V, d, epi=N.EPI_CE_STATS, bias=bias, aux=part, labels=labels,
                                 label_logit=lab),
    }
    for name, fn in cases.items():
        ms = timeit(fn)
        print(f'head M={T} N={V} K={d} epi={name:9s} {ms * 1e3:9.1f} us  {fl / ms / 1e9:7.1f} TF/s', flush=True)


def shape_cases():
    # (M, N, K, a_t, b_t, epi, splits) of the C2 step's main GEMMs
    shapes = [(32768, 512, 32768, 0, 0, N.EPI_BF16, 1),       # head dX (K = V)
              (32768, 512, 32768, 1, 1, N.EPI_F32_ACC, 1),    # head dW (K = T)
              (32768, 2048, 512, 0, 0, N.EPI_BF16, 1),        # FFN1 fwd
              (32768, 512, 2048, 0, 0, N.EPI_F32, 1),         # FFN2 fwd
              (32768, 1536, 512, 0, 0, N.EPI_BF16, 1),        # QKV fwd
              (32768, 512, 512, 0, 0, N.EPI_F32, 1),          # out-proj fwd
              (32768, 2048, 512, 0, 0, N.EPI_BF16, 1),        # FFN2 dX (K = d)
              (32768, 512, 2048, 0, 0, N.EPI_BF16, 1),        # FFN1 dX
              (8192, 8192, 8192, 0, 0, N.EPI_BF16, 1),        # square reference point
              (4096, 4096, 4096, 0, 0, N.EPI_BF16, 1)]
    for (M, N_, K_, at, bt, epi, sp) in shapes:
        A = torch.randn((K_, M) if at else (M, K_), device=dev).to(bf16)
        B = torch.randn((K_, N_) if bt else (N_, K_), device=dev).to(bf16)
        C = torch.zeros(M, N_, device=dev, dtype=f32 if epi in (N.EPI_F32, N.EPI_F32_ACC) else bf16)
        fn = lambda: K.gemm(A, B, C, M, N_, K_, a_t=bool(at), b_t=bool(bt), epi=epi, splits=sp)
        ms = timeit(fn)
        print(f'gemm M={M} N={N_} K={K_} at={at} bt={bt} epi={epi} {ms * 1e3:9.1f} us  '
              f'{2.0 * M * N_ * K_ / ms / 1e9:7.1f} TF/s', flush=True)


def epi_cases():
    """Same shape, different epilogues: the cost of each epilogue over the plain bf16 store."""
    for (M, N_, K_) in [(32768, 512, 2048), (32768, 2048, 512), (32768, 1536, 512)]:
        A = torch.randn(M, K_, device=dev).to(bf16)
        B = torch.randn(N_, K_, device=dev).to(bf16)
        Cb = torch.empty(M, N_, device=dev, dtype=bf16)
        Cf = torch.empty(M, N_, device=dev, dtype=f32)
        R = torch.randn(M, N_, device=dev, dtype=f32)
        aux = torch.randn(M, N_, device=dev).to(bf16)
        bias = torch.randn(N_, device=dev)
        rot = torch.randn(512, 256, 2, device=dev)
        cases = {
            'bf16': lambda: K.gemm(A, B, Cb, M, N_, K_, epi=N.EPI_BF16, bias=bias),
            'f32': lambda: K.gemm(A, B, Cf, M, N_, K_, epi=N.EPI_F32, bias=bias),
            'f32+resid': lambda: K.gemm(A, B, Cf, M, N_, K_, epi=N.EPI_F32, bias=bias, resid=R, ldr=N_),
            'drop+resid': lambda: K.gemm(A, B, Cf, M, N_, K_, epi=N.EPI_DROPOUT_RESID, resid=R, ldr=N_, drop_p=0.1,
                                         seed=5),
            'gelu+aux': lambda: K.gemm(A, B, Cb, M, N_, K_, epi=N.EPI_GELU, bias=bias, aux=aux, ldaux=N_),
            'gelu_bwd': lambda: K.gemm(A, B, Cb, M, N_, K_, epi=N.EPI_GELU_BWD, aux=aux, ldaux=N_),
            'rotary': lambda: K.gemm(A, B, Cb, M, N_, K_, epi=N.EPI_ROTARY_BF16, bias=bias, rot=rot, rot_cols=min(N_, 1024),
                                     rot_d=512, rot_seq=512),
        }
        for name, fn in cases.items():
            ms = timeit(fn)
            print(f'epi M={M} N={N_} K={K_} {name:11s} {ms * 1e3:8.1f} us {2.0 * M * N_ * K_ / ms / 1e9:7.1f} TF/s',
                  flush=True)


if __name__ == '__main__':
    if len(sys.argv) > 1 and sys.argv[1] == 'epi':
        epi_cases()
        sys.exit(0)
    print('SVAE_GEMM_GROUP =', os.environ.get('SVAE_GEMM_GROUP'), 'SVAE_GEMM_EXPT =', os.environ.get('SVAE_GEMM_EXPT'))
    head_cases()
    if len(sys.argv) > 1 and sys.argv[1] == 'all':
        shape_cases()
