"""Time the attention backward at the encoder's shapes (64 learned / latent queries over 512 or 1024 keys, hd 64,
non-causal): one query tile per key block, so each workgroup is mostly prologue and epilogue.

    python scripts/attn_enc_probe.py        (SVAE_ATTN_BWD8=0: the 4-wave 128-key kernel, for A/B)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'sparse-vae_amd'))
import torch  # noqa: E402
from sparse_vae import kernels as K  # noqa: E402

dev = torch.device('cuda', 0)


def timeit(fn, reps=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    for B, H, Lq, Lk, hd, learned in ((64, 8, 64, 512, 64, True), (64, 8, 64, 512, 64, False),
                                      (64, 12, 64, 1024, 64, True), (64, 8, 64, 64, 64, False)):
        d = H * hd
        q = torch.randn(1 if learned else B, Lq, d, device=dev).bfloat16()
        kv = torch.randn(B, Lk, 2 * d, device=dev).bfloat16()
        o = torch.empty(B, Lq, d, device=dev).bfloat16()
        olo = torch.empty_like(o)
        lse = torch.empty(B, H, Lq, device=dev)
        kw = dict(B=B, H=H, Lq=Lq, Lk=Lk, hd=hd, sq=d, bq=0 if learned else Lq * d, sk=2 * d, sv=2 * d, bk=Lk * 2 * d,
                  bv=Lk * 2 * d, so=d, bo=Lq * d, causal=False, o_lo=olo, so_lo=d, bo_lo=Lq * d)
        K.attention(q, kv, kv[:, :, d:], o, lse, **kw)
        dout = torch.randn(B, Lq, d, device=dev).bfloat16()
        dq = torch.empty(B, Lq, d, device=dev)
        dkv = torch.empty(B, Lk, 2 * d, device=dev).bfloat16()
        delta = torch.empty(B, H, Lq, device=dev)
        part = torch.empty(K.attn_dq_part_elems(B, H, Lq, Lk, hd), device=dev)
        bwd = lambda: K.attention(q, kv, kv[:, :, d:], o, lse, backward=True, dout=dout, sdo=d, bdo=Lq * d, delta=delta,  # noqa: E731
                                  dq=dq, bdq=Lq * d, dk=dkv, dv=dkv[:, :, d:], sdk=2 * d, sdv=2 * d, bdk=Lk * 2 * d,
                                  bdv=Lk * 2 * d, dq_part=part, **kw)
        t = timeit(bwd)
        fl = 10.0 * B * H * Lq * Lk * hd
        print(f'B={B} H={H} Lq={Lq} Lk={Lk} hd={hd} learned={int(learned)}  bwd(+delta+dq) {t:7.1f} us '
              f'{fl / t / 1e6:6.1f} TF/s', flush=True)


if __name__ == '__main__':
    main()
