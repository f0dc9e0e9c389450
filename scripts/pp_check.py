"""Bit-exactness of the ping-pong GEMM (SVAE_GEMM_PP=1) against the 256-tile persistent kernel on the shapes it takes:
run `dump` once per setting (the library reads the switch once per process), then `cmp`.

    SVAE_GEMM_PP=0 python scripts/pp_check.py dump /tmp/a.json && SVAE_GEMM_PP=1 python scripts/pp_check.py dump /tmp/b.json
    python scripts/pp_check.py cmp /tmp/a.json /tmp/b.json
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'sparse-vae_amd'))
import torch  # noqa: E402

SHAPES = [(32768, 2048, 512), (32768, 512, 2048), (32768, 1536, 512), (4096, 384, 1024), (65536, 3072, 768),
          (65536, 768, 3072), (512, 256, 576)]


def _hash(t):
    v = t.view(torch.int16).to(torch.int64).flatten()
    w = torch.arange(v.numel(), device=v.device, dtype=torch.int64) % 1000003 + 1
    return int((v * w).sum().item()), int(v.sum().item())


def dump(path):
    from sparse_vae import kernels as K
    from sparse_vae import _native as N
    dev = torch.device('cuda', 0)
    out = {}
    for M, Nn, Kk in SHAPES:
        g = torch.Generator(device='cpu').manual_seed(M + Nn + Kk)
        X = (torch.randn(M, Kk, generator=g) * 0.5).bfloat16().to(dev)
        W = (torch.randn(Nn, Kk, generator=g) * 0.05).bfloat16().to(dev)
        b = torch.randn(Nn, generator=g).to(dev)
        C = torch.empty(M, Nn, device=dev, dtype=torch.bfloat16)
        K.gemm(X, W, C, M, Nn, Kk, epi=N.EPI_BF16, bias=b)
        G = torch.empty(M, Nn, device=dev, dtype=torch.bfloat16)
        Gp = torch.empty(M, Nn, device=dev, dtype=torch.bfloat16)
        K.gemm(X, W, G, M, Nn, Kk, epi=N.EPI_GELU, bias=b, aux=Gp, ldaux=Nn)
        torch.cuda.synchronize()
        ref = (X.float() @ W.float().t() + b)
        err = ((C.float() - ref).norm() / ref.norm()).item()
        out[f'{M}x{Nn}x{Kk}'] = [_hash(C), _hash(G), _hash(Gp), err]
        print(f'{M}x{Nn}x{Kk}: rel err vs fp32 {err:.2e}', flush=True)
    import json
    json.dump(out, open(path, 'w'))


def cmp(a, b):
    import json
    A, B = json.load(open(a)), json.load(open(b))
    ok = True
    for k in A:
        same = A[k][:3] == B[k][:3]
        print(f'{k}: bit-identical {same}')
        ok &= same
    sys.exit(0 if ok else 1)


if __name__ == '__main__':
    if sys.argv[1] == 'dump':
        dump(sys.argv[2])
    else:
        cmp(sys.argv[2], sys.argv[3])
