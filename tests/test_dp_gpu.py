"""The data-parallel path on the GPU with RCCL (backend 'nccl'): a one-rank process group on the box's single GPU
runs the real bucketed async all-reduce overlapped with the engine backward (ready() callbacks, the broadcast at
enable_data_parallel, the final wait). Gradients and the optimizer step must equal the non-DP run (a SUM
all-reduce over one rank; the backward runs on loss / world = loss) up to the backward's own run-to-run noise:
f32 atomics (embedding scatter-add, bias row sums) add in a nondeterministic order, so the bar is 1e-4 of the
norm, not bitwise (measured run-to-run: up to 1.4e-5 of the norm; a DP bug -- a missing 1/world, a bucket reduced
twice or skipped -- is an O(1) relative error). The 2..8-rank runs are the driver's
(bench.py under torch.distributed.run); the multi-rank averaging itself is covered on CPU by test_dp_gloo.py."""
import os
import socket

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu

if torch.cuda.is_available():
    from sparse_vae import TransformerVAE, TransformerVAEHparams, TextDataModule


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model(seed):
    torch.manual_seed(seed)
    hp = TransformerVAEHparams(d_model=256, num_layers=4, num_heads=4, sparse_self_attention=False, kl_weight=0.5)
    m = TransformerVAE(hp, device='cuda')
    m.initialize_weights()
    return m


def test_rccl_data_parallel_one_rank_matches_single_gpu():
    dev = torch.device('cuda', 0)
    dist.init_process_group('nccl', init_method=f'tcp://127.0.0.1:{_port()}', rank=0, world_size=1, device_id=dev)
    try:
        batch = TextDataModule(dataset_name='synthetic', seq_len=256, batch_size=8).synthetic_batch(0, device=dev)
        eps = torch.randn(8, 1, 64, device=dev)
        ref, dp = _model(1), _model(1)
        dp.enable_data_parallel(bucket_mb=4.0)              # small buckets: several all-reduces in flight
        outs = []
        for m in (ref, dp):
            [opt], _ = m.configure_optimizers(8 * 256, 1)
            o = m.training_step(batch, 0, eps=eps, dropout=0.0)
            o['loss'].backward()
            m.on_after_backward()
            g = m._flat.grad[:m._flat.n_live].clone()
            opt.step()
            torch.cuda.synchronize()
            outs.append((o['loss'].item(), g, m._flat.master[:m._flat.n_live].clone()))
        assert outs[0][0] == outs[1][0]
        for a, b in ((outs[0][1], outs[1][1]), (outs[0][2], outs[1][2])):
            assert ((a - b).norm() / b.norm()).item() < 1e-4
    finally:
        dist.destroy_process_group()
