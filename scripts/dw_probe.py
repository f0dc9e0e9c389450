"""Time the weight-gradient GEMMs (C += dY^T X over T tokens) of the C2 step; run under SVAE_GEMM_IMPL=1/2/3 to
compare kernels. python scripts/dw_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'sparse-vae_amd'))
import torch  # noqa: E402
from sparse_vae import kernels as K  # noqa: E402

dev = torch.device('cuda', 0)


def timeit(fn, reps=20):
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


for M, N_, K_ in [(512, 512, 32768), (2048, 512, 32768), (1536, 512, 32768), (512, 2048, 32768), (1024, 512, 32768),
                  (512, 512, 4096)]:
    dY = torch.randn(K_, M, device=dev).to(torch.bfloat16)
    X = torch.randn(K_, N_, device=dev).to(torch.bfloat16)
    C = torch.zeros(M, N_, device=dev)
    bg = torch.zeros(M, device=dev)
    t = timeit(lambda: K.linear_dw(dY, X, C, K_, M, N_, bgrad=bg))
    print(f'impl={os.environ.get("SVAE_GEMM_IMPL", "auto")} dW M={M} N={N_} K={K_} splits={K.auto_splits(M, N_, K_)} '
          f'{t:7.1f} us {2.0 * M * N_ * K_ / t / 1e6:7.1f} TF/s', flush=True)

# the two paired launches of the step (FFN1 + FFN2 weight gradients; QKV + out-projection with their bias sums)
T, d = 32768, 512
h = torch.randn(T, d, device=dev).to(torch.bfloat16)
dY2 = torch.randn(T, 2048, device=dev).to(torch.bfloat16)
dq = torch.randn(T, 1536, device=dev).to(torch.bfloat16)
Wg1, Wg2 = torch.zeros(2048, d, device=dev), torch.zeros(d, 2048, device=dev)
Wq, Wo, bq, bo = torch.zeros(1536, d, device=dev), torch.zeros(d, d, device=dev), torch.zeros(1536, device=dev), \
    torch.zeros(d, device=dev)
t = timeit(lambda: K.linear_dw_pair((dY2, h, Wg1, T, 2048, d, None, None, None), (h, dY2, Wg2, T, d, 2048, None, None,
                                                                                  None)))
print(f'pair ffn1+ffn2 dW {t:7.1f} us {2.0 * 2 * 2048 * d * T / t / 1e6:7.1f} TF/s', flush=True)
t = timeit(lambda: K.linear_dw_pair((dq, h, Wq, T, 1536, d, None, None, bq), (h, h, Wo, T, d, d, None, None, bo)))
print(f'pair qkv+out dW (bias sums) {t:7.1f} us {2.0 * (1536 + 512) * d * T / t / 1e6:7.1f} TF/s', flush=True)
t = timeit(lambda: K.linear_dw_pair((dq, h, Wq, T, 1536, d, None, None, None), (h, h, Wo, T, d, d, None, None, None)))
print(f'pair qkv+out dW (no bias) {t:7.1f} us {2.0 * (1536 + 512) * d * T / t / 1e6:7.1f} TF/s', flush=True)
