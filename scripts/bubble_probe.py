"""GPU-side cost of a launch: 200 tiny kernels (4-byte adds) and 200 of our smallest library kernel captured in one HIP
graph and replayed; per-launch time = replay time / 200 (no host launch cost in a replay)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'sparse-vae_amd'))
import torch  # noqa: E402
from sparse_vae import kernels as K  # noqa: E402

dev = torch.device('cuda', 0)
x = torch.zeros(1, device=dev)
part = torch.zeros(64, device=dev)
g32 = torch.randn(4096, device=dev)


def graph_time(fn, n=200, reps=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (reps * n)


print(f'torch add_ (1 element): {graph_time(lambda: x.add_(1.0)):.2f} us per launch in a graph', flush=True)
print(f'svae_sumsq (4096 floats, 4 blocks): {graph_time(lambda: K.sumsq(g32, 4096, part[:4])):.2f} us per launch in a graph', flush=True)
