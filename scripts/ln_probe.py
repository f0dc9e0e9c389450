"""LayerNorm forward timing at the C2 / C4 row shapes (f32 in, bf16 out), 50 back-to-back launches, with an exactness
check against torch (f32 LayerNorm, then bf16). SVAE_LN_FWD_BLOCKS selects the grid cap (0: one row per wave).

    SVAE_LN_FWD_BLOCKS=1024 python scripts/ln_probe.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'sparse-vae_amd'))
import torch  # noqa: E402
from sparse_vae import kernels as K  # noqa: E402

dev = torch.device('cuda', 0)
cap = os.environ.get('SVAE_LN_FWD_BLOCKS', 'default')
for rows, D in ((32768, 512), (4096, 512), (65536, 768), (8192, 768), (1000, 1024), (777, 760)):
    x = torch.randn(rows, D, device=dev)
    w = torch.randn(D, device=dev)
    b = torch.randn(D, device=dev)
    y = torch.empty(rows, D, device=dev, dtype=torch.bfloat16)
    mean = torch.empty(rows, device=dev)
    rstd = torch.empty(rows, device=dev)
    K.layernorm_fwd(x, w, b, y, mean, rstd, rows, D)
    ref = torch.nn.functional.layer_norm(x, (D,), w, b, 1e-5)
    err = ((y.float() - ref).abs() / (ref.abs() + 1e-2)).max().item()
    for _ in range(3):
        K.layernorm_fwd(x, w, b, y, mean, rstd, rows, D)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        K.layernorm_fwd(x, w, b, y, mean, rstd, rows, D)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 50
    gbs = rows * D * 6 / us / 1e3
    print(f'cap {cap:>7s} rows {rows:6d} D {D:4d}: {us:7.2f} us  {gbs:7.1f} GB/s  max rel err {err:.2e}', flush=True)
    assert err < 1e-2, err
