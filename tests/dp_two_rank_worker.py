"""Worker of tests/test_dp_gpu_2rank.py (not collected by pytest): one data-parallel rank of the real GPU training
step. Both ranks run on the box's single GPU with the gloo backend (RCCL allows one rank per GPU); the model's
bucketed async all-reduces, the engine's ready() callbacks and the 1/world scaling are the code the N-GPU run uses.

    python tests/dp_two_rank_worker.py RANK WORLD PORT OUT.pt
Rank r trains on sequences [r*B/world, (r+1)*B/world) of one synthetic batch; rank 0 also runs the same step without
data parallelism on the whole batch (the reference the averaged gradient must equal)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'sparse-vae_amd'))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from sparse_vae import TransformerVAE, TransformerVAEHparams, TextDataModule  # noqa: E402
from sparse_vae.core.padded_tensor import PaddedTensor  # noqa: E402

B, L = 8, 128


def _model(seed):
    torch.manual_seed(seed)
    hp = TransformerVAEHparams(d_model=256, num_layers=4, num_heads=4, sparse_self_attention=False, kl_weight=0.5)
    m = TransformerVAE(hp, device='cuda')
    m.initialize_weights()
    return m


def _slice(batch, lo, hi):
    raw = batch['token_ids'].as_raw()[lo:hi]
    return {'token_ids': PaddedTensor.from_raw(raw.contiguous()), 'num_tokens': batch['num_tokens'][lo:hi].contiguous(),
            'num_bytes': batch['num_bytes'][lo:hi].contiguous()}


def _step(m, batch, eps):
    o = m.training_step(batch, 0, eps=eps, dropout=0.0)
    o['loss'].backward()
    torch.cuda.synchronize()
    return o['loss'].item(), m._flat.grad[:m._flat.n_live].detach().cpu().clone()


def main():
    rank, world, port, out = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    dist.init_process_group('gloo', init_method=f'tcp://127.0.0.1:{port}', rank=rank, world_size=world)
    batch = TextDataModule(dataset_name='synthetic', seq_len=L, batch_size=B).synthetic_batch(0, device=dev)
    gen = torch.Generator().manual_seed(7)
    eps = torch.randn(B, 1, 64, generator=gen).to(dev)
    per = B // world
    m = _model(1 + rank)                     # different init per rank: enable_data_parallel broadcasts rank 0's
    m.enable_data_parallel(bucket_mb=1.0)    # small buckets: many all-reduces in flight during the backward
    loss, g = _step(m, _slice(batch, rank * per, (rank + 1) * per), eps[rank * per:(rank + 1) * per])
    res = {'rank': rank, 'loss': loss, 'grad': g, 'w': m._flat.master[:4096].detach().cpu().clone()}
    if rank == 0:
        ref = _model(1)
        res['ref_loss'], res['ref_grad'] = _step(ref, batch, eps)
    # gradient accumulation under DP (accumulate_grad_batches = 2, DDP no_sync): two micro-steps of per / 2 sequences;
    # the first reduces nothing, the second's buckets reduce the accumulated sum once
    m.zero_grad()
    q = per // 2
    for k, sync in ((0, False), (1, True)):
        lo = rank * per + k * q
        m.require_backward_grad_sync = sync
        o = m.training_step(_slice(batch, lo, lo + q), 0, eps=eps[lo:lo + q], dropout=0.0)
        o['loss'].backward()
        if not sync:
            assert not m._dp['works'] and m._dp['start'] == 0, 'a no_sync micro-step communicated'
    torch.cuda.synchronize()
    res['acc_grad'] = m._flat.grad[:m._flat.n_live].detach().cpu().clone()
    if rank == 0:
        # single process, no DP: micro-batch k = the ranks' k-th micro-batches together (a mean over 2q sequences of
        # equal length = the rank mean of the q-sequence means), gradients accumulated over the two micro-steps
        ref.zero_grad()
        raw = batch['token_ids'].as_raw()
        for k in (0, 1):
            idx = torch.tensor([r * per + k * q + j for r in range(world) for j in range(q)], device=dev)
            sub = {'token_ids': PaddedTensor.from_raw(raw[idx].contiguous()),
                   'num_tokens': batch['num_tokens'][idx].contiguous(), 'num_bytes': batch['num_bytes'][idx].contiguous()}
            ref.training_step(sub, 0, eps=eps[idx], dropout=0.0)['loss'].backward()
        torch.cuda.synchronize()
        res['ref_acc_grad'] = ref._flat.grad[:ref._flat.n_live].detach().cpu().clone()
    torch.save(res, out)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
