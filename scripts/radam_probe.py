"""Fused clip + RAdam kernel alone at the C2 / C4 parameter counts (46 M / 162 M f32 parameters): time per launch
(20 back-to-back) and the effective bandwidth at 30 B per parameter; checked against a torch restatement of the
update for one launch."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'sparse-vae_amd'))
import torch  # noqa: E402
from sparse_vae import kernels as K  # noqa: E402

dev = torch.device('cuda', 0)
for n in (46_000_000, 162_000_000):
    g = torch.randn(n, device=dev) * 1e-3
    m = torch.randn(n, device=dev) * 1e-4
    v = torch.rand(n, device=dev) * 1e-6
    p = torch.randn(n, device=dev)
    pbf = torch.empty(n, device=dev, dtype=torch.bfloat16)
    part = torch.zeros(1024, device=dev)
    K.sumsq(g, n, part)
    # scal: lr_eff, bcm, bcv, rho_ok, beta1, beta2, eps, wd, max_norm
    scal = torch.tensor([3e-4, 0.1, 0.3, 1.0, 0.9, 0.999, 1e-8, 0.0, 150.0], device=dev)
    m0, v0, p0 = m.clone(), v.clone(), p.clone()
    K.radam(p, pbf, g, m, v, n, part, scal, None)
    torch.cuda.synchronize()
    norm = g.double().norm().item()
    coef = min(1.0, 150.0 / (norm + 1e-6))
    gi = g * coef
    mr = m0 * 0.9 + 0.1 * gi
    vr = v0 * 0.999 + 0.001 * gi * gi
    pr = p0 - (3e-4 / 0.1) * (mr / (vr.sqrt() / 0.3 + 1e-8))
    err = max((m - mr).abs().max().item(), (v - vr).abs().max().item() * 1e3, (p - pr).abs().max().item())
    for _ in range(3):
        K.radam(p, pbf, g, m, v, n, part, scal, None)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        K.radam(p, pbf, g, m, v, n, part, scal, None)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 20
    print(f'n {n / 1e6:6.1f} M: radam {us:7.1f} us  {30 * n / us / 1e3:6.1f} GB/s  max err {err:.2e}', flush=True)
    assert err < 1e-5, err
    del g, m, v, p, pbf, m0, v0, p0, mr, vr, pr, gi
