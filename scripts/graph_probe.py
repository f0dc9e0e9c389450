"""How much of the eager C2 step is launch / inter-kernel overhead: the bench step timed eagerly, then the same step
captured once into a HIP graph and replayed (host-side scalars -- seeds, the RAdam step and LR -- frozen at capture,
so this is a timing probe, not a training mode).

    python scripts/graph_probe.py [c2] [steps]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'sparse-vae_amd'))
import torch  # noqa: E402
import bench  # noqa: E402


def main():
    cfg_name = sys.argv[1] if len(sys.argv) > 1 else 'c2'
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device('cuda', 0)
    model, opt, sch, batch = bench.build(bench.CONFIGS[cfg_name], dev)
    for _ in range(3):
        bench.step(model, opt, sch, batch)
    torch.cuda.synchronize()

    def timed(fn, n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / n

    import sparse_vae.transformer_vae as tv
    normal = tv.Normal
    tv.Normal = lambda loc, scale, validate_args=None: normal(loc, scale, validate_args=True)   # noqa: E731
    eager_sync = timed(lambda: bench.step(model, opt, sch, batch), steps)
    tv.Normal = normal
    eager = timed(lambda: bench.step(model, opt, sch, batch), steps)
    print(f'{cfg_name} eager, posterior validated (host sync) {eager_sync:7.3f} ms/step; eager {eager:7.3f} ms/step',
          flush=True)
    # CPU time per eager step with the GPU not waited for: the launch cost the host pays
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    bench.step(model, opt, sch, batch)
    host = (time.perf_counter() - t0) * 1e3
    torch.cuda.synchronize()
    print(f'{cfg_name} host time of one eager step (no sync) {host:7.3f} ms', flush=True)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            bench.step(model, opt, sch, batch)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        bench.step(model, opt, sch, batch)
    torch.cuda.synchronize()
    for _ in range(3):
        g.replay()
    graph = timed(g.replay, steps)
    print(f'{cfg_name} graph  {graph:7.3f} ms/step  ({100 * (eager - graph) / eager:+.1f} % of the eager step)',
          flush=True)


if __name__ == '__main__':
    main()
