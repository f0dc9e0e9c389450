"""Time the fused clip + RAdam update alone (svae_radam) at the C2 and C4 parameter counts; 30 B per parameter moved
(read g, m, v, p; write m, v, p, bf16 shadow). Variants through SVAE_RADAM_U / _NT / _GRID.

    python scripts/radam_probe.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'sparse-vae_amd'))
import torch  # noqa: E402
from sparse_vae import kernels as K  # noqa: E402

dev = torch.device('cuda', 0)


def main():
    for n in (45_000_000, 162_000_000):
        p = torch.randn(n, device=dev)
        g = torch.randn(n, device=dev) * 1e-3
        m = torch.zeros(n, device=dev)
        v = torch.zeros(n, device=dev)
        pbf = torch.empty(n, device=dev, dtype=torch.bfloat16)
        part = torch.empty(1024, device=dev)
        K.sumsq(g, n, part)
        scal = torch.tensor([1e-4, 0.1, 0.01, 1.0, 0.9, 0.999, 1e-8, 0.0, 1e9], device=dev)
        norm = torch.empty(1, device=dev)
        fn = lambda: K.radam(p, pbf, g, m, v, n, part, scal, norm)  # noqa: E731
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / 20 * 1e3
        print(f'n={n / 1e6:6.1f} M  {t:8.1f} us  {30 * n / t / 1e3:7.1f} GB/s', flush=True)


if __name__ == '__main__':
    main()
