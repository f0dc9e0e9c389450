"""The bf16 noise floor of the step-parity test's gradient bars (verdict r05 item 4), on CPU.

The GPU step computes every GEMM and attention product on bf16 operands (f32 accumulation); the test compares it with
the fp32 oracle per parameter (cosine >= 0.995, norm ratio within 2 % / 5 %). How far apart may two CORRECT bf16
implementations land? Here the oracle (pinned to the reference by tests/golden) runs at a golden configuration in
  * fp64 (the truth),
  * fp32 (what the test compares against),
  * bf16-operand emulations: every matmul / F.linear of the forward AND of its backward takes its operands rounded
    to bf16 (round-to-nearest, plus NSR stochastic-rounding draws), accumulating in the working precision -- the
    GPU's numerics model without its particular summation orders;
and reports, per parameter, each run's gradient cosine and norm ratio against fp64. The stochastic-rounding draws'
spread of the norm ratio is the per-parameter noise floor: a correct bf16 implementation sits inside it, and a bar
drawn at a stated multiple of it separates a regression from rounding.

    python scripts/noise_floor.py c4shape [--nsr 4] [--out profiles/r06_noise_floor_c4shape.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.nn.functional as F
from torch.overrides import TorchFunctionMode

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import oracle  # noqa: E402
from golden_util import setup  # noqa: E402


class _Round:
    """bf16 rounding of an operand: round-to-nearest-even, or stochastic (add 16 random low bits, truncate)."""

    def __init__(self, seed=None):
        self.gen = None if seed is None else torch.Generator().manual_seed(seed)

    def __call__(self, x):
        if self.gen is None:
            return x.to(torch.bfloat16).to(x.dtype)
        x32 = x.float().contiguous()
        bits = x32.view(torch.int32)
        r = torch.randint(0, 1 << 16, bits.shape, generator=self.gen, dtype=torch.int32)
        out = ((bits + r) & ~0xFFFF).view(torch.float32)
        return out.to(x.dtype)


class _BMM(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b, rnd):
        ctx.save_for_backward(a, b)
        ctx.rnd = rnd
        return torch.matmul(rnd(a), rnd(b))

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        rnd = ctx.rnd
        gr = rnd(g)
        ga = torch.matmul(gr, rnd(b).transpose(-1, -2))
        gb = torch.matmul(rnd(a).transpose(-1, -2), gr)
        # broadcast reductions (a batched operand against an unbatched one)
        while ga.dim() > a.dim():
            ga = ga.sum(0)
        while gb.dim() > b.dim():
            gb = gb.sum(0)
        for i, (sa, sg) in enumerate(zip(a.shape, ga.shape)):
            if sa == 1 and sg != 1:
                ga = ga.sum(i, keepdim=True)
        for i, (sb, sg) in enumerate(zip(b.shape, gb.shape)):
            if sb == 1 and sg != 1:
                gb = gb.sum(i, keepdim=True)
        return ga, gb, None


class Bf16Operands(TorchFunctionMode):
    """Every matmul / linear of the oracle on bf16-rounded operands (forward and backward)."""

    def __init__(self, rnd):
        super().__init__()
        self.rnd = rnd

    def __torch_function__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if func in (torch.matmul, torch.Tensor.__matmul__):
            return _BMM.apply(args[0], args[1], self.rnd)
        if func is F.linear:
            x, w = args[0], args[1]
            b = args[2] if len(args) > 2 else kwargs.get('bias')
            y = _BMM.apply(x, w.t(), self.rnd)
            return y + b if b is not None else y
        return func(*args, **kwargs)


def run(name, dtype, mode=None):
    g, hp, params, ids = setup(name)
    ntok = torch.from_numpy(g['lens'])
    eps = torch.from_numpy(g['eps']).to(dtype)
    p = {k: v.to(dtype).clone().requires_grad_(True) for k, v in params.items()}
    t0 = time.time()
    if mode is None:
        ref = oracle.training_step(p, hp, ids, ntok, eps, kl_weight=float(g['kl_weight']))
        ref['loss'].backward()
    else:
        with mode:
            ref = oracle.training_step(p, hp, ids, ntok, eps, kl_weight=float(g['kl_weight']))
        ref['loss'].backward()
    grads = {k: v.grad.detach().double().flatten() for k, v in p.items() if v.grad is not None}
    return ref['loss'].item(), grads, time.time() - t0


def compare(grads, truth):
    out = {}
    for n, t in truth.items():
        gg = grads[n]
        out[n] = ((gg @ t / (gg.norm() * t.norm() + 1e-300)).item(), (gg.norm() / (t.norm() + 1e-300)).item())
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('name', nargs='?', default='c4shape')
    ap.add_argument('--nsr', type=int, default=4)
    ap.add_argument('--threads', type=int, default=min(16, os.cpu_count()))
    ap.add_argument('--out', default=None)
    args = ap.parse_args()
    torch.set_num_threads(args.threads)
    loss64, g64, t = run(args.name, torch.float64)
    print(f'fp64 loss {loss64:.9f} ({t:.0f} s)', flush=True)
    runs = {}
    loss32, g32, t = run(args.name, torch.float32)
    runs['fp32'] = (loss32, compare(g32, g64))
    print(f'fp32 loss {loss32:.9f} ({t:.0f} s)', flush=True)
    lr, gr, t = run(args.name, torch.float32, Bf16Operands(_Round()))
    runs['bf16_rn'] = (lr, compare(gr, g64))
    print(f'bf16 round-to-nearest loss {lr:.9f} ({t:.0f} s)', flush=True)
    for s in range(args.nsr):
        ls, gs, t = run(args.name, torch.float32, Bf16Operands(_Round(seed=100 + s)))
        runs[f'bf16_sr{s}'] = (ls, compare(gs, g64))
        print(f'bf16 stochastic #{s} loss {ls:.9f} ({t:.0f} s)', flush=True)

    names = list(g64.keys())
    sr = [k for k in runs if k.startswith('bf16')]
    table = {}
    for n in names:
        ratios = np.array([runs[k][1][n][1] for k in sr])
        coss = np.array([runs[k][1][n][0] for k in sr])
        table[n] = {'fp32_cos': runs['fp32'][1][n][0], 'fp32_ratio': runs['fp32'][1][n][1],
                    'bf16_ratio_dev_max': float(np.abs(ratios - 1).max()), 'bf16_ratio_std': float(ratios.std()),
                    'bf16_cos_min': float(coss.min())}
    worst = sorted(names, key=lambda n: -table[n]['bf16_ratio_dev_max'])
    print(f'{"parameter":58s} fp32 |r-1|  bf16 max|r-1|  bf16 std(r)  bf16 min cos')
    for n in worst[:20]:
        t_ = table[n]
        print(f'{n:58s} {abs(t_["fp32_ratio"] - 1):10.2e} {t_["bf16_ratio_dev_max"]:13.4f} {t_["bf16_ratio_std"]:11.4f} '
              f'{t_["bf16_cos_min"]:12.5f}')
    if args.out:
        with open(args.out, 'w') as f:
            json.dump({'config': args.name, 'source': 'scripts/noise_floor.py (CPU oracle, fp64 truth)',
                       'loss': {'fp64': loss64, **{k: v[0] for k, v in runs.items()}},
                       'runs': sr, 'per_parameter': table}, f, indent=1)


if __name__ == '__main__':
    main()
