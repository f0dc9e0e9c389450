"""8192^3 bf16 GEMM launches of libsvae (the gemm256 kernel, bf16 epilogue) for the SQ-counter calibration of
scripts/pmc_gemm_sq.sh: 2 warm-up launches, then 5; prints the HIP-event average and TF/s."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'sparse-vae_amd'))
import torch  # noqa: E402
from sparse_vae import kernels as K  # noqa: E402
from sparse_vae import _native as N  # noqa: E402

dev = torch.device('cuda', 0)
n = 8192
a = torch.randn(n, n, device=dev).bfloat16()
w = torch.randn(n, n, device=dev).bfloat16()
c = torch.empty(n, n, device=dev, dtype=torch.bfloat16)
for _ in range(2):
    K.gemm(a, w, c, n, n, n, epi=N.EPI_BF16)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(5):
    K.gemm(a, w, c, n, n, n, epi=N.EPI_BF16)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 5
print(f'gemm 8192^3 bf16: {ms * 1e3:.1f} us per launch, {2 * n ** 3 / ms / 1e9:.1f} TF/s', flush=True)
