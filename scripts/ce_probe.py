"""Time ce_grad alone at the C2 head shape (32K tokens x 32K vocab, bf16 logits in place) against an in-place
torch read+write of the same buffer. SVAE_LIB selects an A/B build."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'sparse-vae_amd'))
from sparse_vae import kernels as K  # noqa: E402


def timeit(fn, n=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


rows, V, seq = 32768, 32768, 512
dev = 'cuda'
logits = (torch.randn(rows, V, device=dev) * 0.1).to(torch.bfloat16)
lse = torch.full((rows,), 10.4, device=dev)
chunk_w = torch.ones(1, device=dev)
labels = torch.randint(3, V, (rows,), device=dev, dtype=torch.int32)
g = torch.full((1,), 1.0 / rows, device=dev)
dbias = torch.zeros(V, device=dev)
for name, db in (('with dbias', dbias), ('no dbias', None)):
    us = timeit(lambda: K.ce_grad(logits, V, lse, chunk_w, labels, g, rows, V, seq, 1, seq, dbias=db))
    print(f'{os.environ.get("SVAE_LIB", "default")}: ce_grad {name}: {us:.1f} us = {4 * rows * V / us / 1e6:.2f} TB/s')
us = timeit(lambda: logits.mul_(1.0))
print(f'torch in-place mul_ (same bytes): {us:.1f} us = {4 * rows * V / us / 1e6:.2f} TB/s')
