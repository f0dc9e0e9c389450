"""Throughput of the evaluation and generation paths on one MI355X (secondary to bench.py's training metric).

    python scripts/bench_eval.py [--batch 64] [--seq 512] [--gen-len 512]

* IW-NLL: TransformerVAE.test_step (transformer_vae.py:71-79: q(z|x), 100 posterior samples, log p(x|z) per
  sample through the batched bf16 decoder + stats-only vocabulary GEMM) on the C2 model; tokens/s counts the
  decoded tokens (100 * B * L).
* Generation: TransformerVAE.sample (greedy and nucleus, KV cache, f32 decode kernels) at batch B for
  gen-len positions, HIP-graph replay vs eager launches; tokens/s = B * steps / time.
Random-init weights, synthetic ids (the decode runs to max length: no end token is produced).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'sparse-vae_amd'))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=64)
    ap.add_argument('--seq', type=int, default=512)
    ap.add_argument('--gen-len', type=int, default=512)
    ap.add_argument('--gen-batch', type=int, default=64)
    a = ap.parse_args()
    from sparse_vae import TransformerVAE, TransformerVAEHparams, TextDataModule
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    hp = TransformerVAEHparams(d_model=512, num_layers=6, num_heads=8, latent_depth=64, sparse_self_attention=False,
                               kl_weight=1.0)
    model = TransformerVAE(hp, device=dev)
    model.initialize_weights()
    model.eval()
    res = {}
    batch = TextDataModule(dataset_name='synthetic', seq_len=a.seq, batch_size=a.batch).synthetic_batch(0, device=dev)
    model.test_step(batch, 0)                                    # warm-up (workspaces)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    reps = 3
    for _ in range(reps):
        nll = model.test_step(batch, 0)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    res['iw_nll'] = {'batch': a.batch, 'seq_len': a.seq, 'samples': 100, 's_per_test_step': round(dt, 4),
                     'decoded_tokens_per_s': round(100 * a.batch * a.seq / dt, 1), 'nll_iw': round(nll.item(), 5)}
    print(json.dumps(res['iw_nll']), flush=True)
    model.end_token = -1                                          # never stops early: full-length decode
    for mode, kw in (('greedy', dict(temperature=0.0)), ('nucleus', dict(temperature=1.0, top_p=0.9))):
        for graph in (True, False):
            z = torch.randn(a.gen_batch, 1, 64, device=dev)
            model.sample(8, a.gen_batch, z=z, use_graph=graph, **kw)           # warm-up
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = model.sample(a.gen_len, a.gen_batch, z=z, use_graph=graph, **kw)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            steps = a.gen_len - 2
            r = {'mode': mode, 'graph': graph, 'batch': a.gen_batch, 'max_length': a.gen_len,
                 'ms_per_step': round(dt / steps * 1e3, 4), 'tokens_per_s': round(a.gen_batch * steps / dt, 1),
                 'nonzero_ids': int((out != 0).sum().item())}
            res[f'sample_{mode}_{"graph" if graph else "eager"}'] = r
            print(json.dumps(r), flush=True)


if __name__ == '__main__':
    main()
