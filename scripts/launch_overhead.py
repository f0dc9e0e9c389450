"""Fixed cost of a gemm256 launch outside its blocks' lifetimes: HIP-event time of one launch and the mean of 20
back-to-back launches, for a 1-tile GEMM and the one-tile-per-CU K = 64 / 512 shapes, beside torch memsets.
With the stamps build the blocks' entry/exit on the 100 MHz clock are printed too.

    SVAE_GEMM_IMPL=3 SVAE_LIB=sparse-vae_amd/sparse_vae/libsvae_stamps.so python scripts/launch_overhead.py
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'sparse-vae_amd'))
import torch  # noqa: E402
from sparse_vae import kernels as K  # noqa: E402
from sparse_vae import _native as N  # noqa: E402

dev = torch.device('cuda', 0)
bf16 = torch.bfloat16
has_rt = hasattr(N.lib, 'svae_debug_rt')


def ev(fn, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def rt(nblk):
    buf = np.zeros((1024, 2), dtype=np.uint64)
    N.lib.svae_debug_rt.argtypes = [ctypes.c_void_p]
    assert N.lib.svae_debug_rt(buf.ctypes.data) == 0
    b = buf[:nblk].astype(np.int64)
    t0 = b[:, 0].min()
    return f'blocks live {(b[:, 1].max() - t0) / 100:5.1f} us'


h = torch.randn(32768, 512, device=dev).to(bf16)
W = (0.02 * torch.randn(512, 512, device=dev)).to(bf16)
ob = torch.empty(32768, 512, device=dev, dtype=bf16)
o32 = torch.empty(32768, 512, device=dev)
cases = [
    ('1 tile 256x256 K64', lambda: K.gemm(h[:256, :64], W[:256, :64], ob[:256, :256], 256, 256, 64, lda=512, ldb=512,
                                          ldc=512), 1),
    ('1 tile 256x256 K512', lambda: K.gemm(h[:256], W[:256], ob[:256, :256], 256, 256, 512, ldc=512), 1),
    ('8 tiles K512', lambda: K.gemm(h[:1024], W, ob[:1024], 1024, 512, 512), 8),
    ('256 tiles K64', lambda: K.gemm(h[:, :64], W[:, :64], ob, 32768, 512, 64, lda=512, ldb=512), 256),
    ('256 tiles K512 bf16', lambda: K.gemm(h, W, ob, 32768, 512, 512), 256),
    ('256 tiles K512 f32', lambda: K.gemm(h, W, o32, 32768, 512, 512, epi=N.EPI_F32), 256),
    ('memset 32 MB', lambda: ob.zero_(), 0),
    ('memset 64 MB', lambda: o32.zero_(), 0),
    ('empty-ish add 4 B', lambda: o32[:1, :1].add_(1.0), 0),
]
for name, fn, nb in cases:
    for _ in range(3):
        fn()
    one = ev(fn, 1)
    extra = rt(nb) if has_rt and nb else ''
    many = ev(fn, 20)
    print(f'{name:22s} single {one:6.1f} us  back-to-back {many:6.1f} us  {extra}', flush=True)
