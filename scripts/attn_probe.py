"""Time the flash attention kernels alone at the C2 decoder shape (B=64, H=8, L=512, hd=64, q|k|v interleaved),
some neighbours, and the C4 decoder shape (L=1024, hd=96).

    python scripts/attn_probe.py
ATTN_PROBE_ONLY: hd96 | c2c4 | c2c4c5 (adds the C5 decoder shape B=32, L=2048, hd 96); ATTN_PROBE_ROT=1: the backward
with the inverse rotary fused (bf16 dQ with rotary, as the engine runs it).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'sparse-vae_amd'))
import torch  # noqa: E402
from sparse_vae import kernels as K  # noqa: E402
from sparse_vae.engine import rotary_table  # noqa: E402

dev = torch.device('cuda', 0)


def timeit(fn, reps=20):
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
    only = os.environ.get('ATTN_PROBE_ONLY')   # e.g. 'hd96': only the C4 decoder shape
    cases = [(64, 512, True, 64), (64, 512, False, 64), (16, 512, True, 64), (256, 512, True, 64), (64, 1024, True, 64),
             (64, 1024, True, 96), (32, 2048, True, 96)]
    rot_on = os.environ.get('ATTN_PROBE_ROT') == '1'
    for B, L, causal, hd in cases:
      if only == 'hd96' and hd != 96:
          continue
      if only == 'c2c4' and (B, L, causal, hd) not in ((64, 512, True, 64), (64, 1024, True, 96)):
          continue
      if only == 'c2c4c5' and (B, L, causal, hd) not in ((64, 512, True, 64), (64, 1024, True, 96), (32, 2048, True, 96)):
          continue
      if not only and L == 2048:
          continue
      for with_o32 in (True, 'olo', False):
        H = 8
        if with_o32 is not True and (B, L, hd) != (64, 512, 64) and not only:
            continue
        d = H * hd
        qkv = torch.randn(B * L, 3 * d, device=dev).bfloat16()
        o = torch.empty(B * L, d, device=dev).bfloat16()
        o32 = torch.empty(B * L, d, device=dev)
        lse = torch.empty(B, H, L, device=dev)
        olo = torch.empty(B * L, d, device=dev).bfloat16()
        kw = dict(B=B, H=H, Lq=L, Lk=L, hd=hd, sq=3 * d, sk=3 * d, sv=3 * d, so=d, bq=L * 3 * d, bk=L * 3 * d,
                  bv=L * 3 * d, bo=L * d, causal=causal, o32=o32 if with_o32 is True else None, so32=d, bo32=L * d,
                  o_lo=olo if with_o32 == 'olo' else None, so_lo=d, bo_lo=L * d)
        fwd = lambda: K.attention(qkv, qkv[:, d:], qkv[:, 2 * d:], o, lse, **kw)
        t = timeit(fwd)
        fl = 4.0 * B * H * L * L * hd * (0.5 if causal else 1.0)
        dout = torch.randn(B * L, d, device=dev).bfloat16()
        dqkv = torch.empty(B * L, 3 * d, device=dev).bfloat16()
        delta = torch.empty(B, H, L, device=dev)
        part = torch.empty(K.attn_dq_part_elems(B, H, L, L, hd), device=dev)
        rkw = dict(rot=rotary_table(L, d).to(dev), rot_d=d) if rot_on else {}
        bwd = lambda: K.attention(qkv, qkv[:, d:], qkv[:, 2 * d:], o, lse, backward=True, dout=dout, sdo=d, bdo=L * d,
                                  delta=delta, dq_bf=dqkv, ldq_bf=3 * d, dk=dqkv[:, d:], dv=dqkv[:, 2 * d:], sdk=3 * d,
                                  sdv=3 * d, bdk=L * 3 * d, bdv=L * 3 * d, dq_part=part, **rkw, **kw)
        if not with_o32:
            print(f'B={B:4d} L={L:5d} hd={hd:3d} causal={int(causal)} no-o32 fwd {t:8.1f} us', flush=True)
            continue
        tb = timeit(bwd)
        tag = 'o32' if with_o32 is True else 'olo'
        print(f'B={B:4d} L={L:5d} hd={hd:3d} causal={int(causal)} {tag} fwd {t:8.1f} us {fl / t / 1e6:7.1f} TF/s   '
              f'bwd(+delta+dq) {tb:8.1f} us {2.5 * fl / tb / 1e6:7.1f} TF/s', flush=True)


if __name__ == '__main__':
    main()
