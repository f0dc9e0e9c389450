"""TransformerVAE (transformer_vae.py:16-128 in the reference) on MI355X.

Same hparams dataclass, module tree and `state_dict` keys as the reference; the arithmetic of
`training_step` / `reconstruct` runs in the fused HIP step engine (sparse_vae/engine.py). Parameters are
views into one flat f32 arena (+ bf16 shadow, + flat grad arena) in gradient-ready order.

Autograd compatibility: `training_step` returns a loss tensor whose `.backward()` runs the engine's
explicit backward and leaves every parameter's `.grad` as a view of the gradient arena, so the reference's
Lightning loop (training_step -> backward -> on_after_backward -> optimizer.step) works unchanged.
"""
import math
import os
import warnings
from copy import deepcopy
from dataclasses import dataclass
from typing import Any, Dict, Optional

import torch
import torch.distributed as dist
from torch import nn
from torch.distributions.normal import Normal

from .core import (ContinuousVAEHparams, ContinuousVAEHooks, ConditionalGaussian, LanguageModel, Perceiver,
                   TransformerHparams, TransformerLayer, VOCAB_SIZE)
from .core.padded_tensor import PaddedTensor
from .engine import FlatParams, VAEEngine
from .core.generation import GenerationState
from .decoding import KVDecoder
from . import kernels as K
from ._native import EPI_F32, EPI_BF16


@dataclass
class TransformerVAEHparams(TransformerHparams, ContinuousVAEHparams):
    latent_depth: int = 64
    pretrained_encoder: bool = False
    pretrained_decoder: bool = False
    use_gpt2: bool = False
    early_stopping_metric: str = 'val_nll'


class _EngineHP:
    """The view of the hparams the engine reads."""

    def __init__(self, hp):
        self.d_model, self.num_heads, self.num_layers = hp.d_model, hp.num_heads, hp.num_layers
        self.latent_depth, self.num_latents, self.vocab_size = hp.latent_depth, 64, VOCAB_SIZE
        self.enc_layers = hp.num_layers // 2
        # decoder self-attention: 0 = dense, else SparseAttention's window in 32-token blocks
        # (transformer_language_model.py:67-69 passes attn_window_size when sparse_self_attention)
        self.attn_window = int(hp.get('attn_window_size', 4)) if hp.get('sparse_self_attention', True) else 0


class _StepFn(torch.autograd.Function):
    """One autograd node for the whole step: backward = the engine's explicit backward."""

    @staticmethod
    def forward(ctx, anchor, model, loss):
        ctx.model = model
        return loss.detach().clone()

    @staticmethod
    def backward(ctx, gloss):
        ctx.model._run_backward(gloss)
        return None, None, None


class TransformerVAE(ContinuousVAEHooks, LanguageModel):
    def __init__(self, hparams, device: Optional[str] = None):
        super().__init__(hparams)
        hp = self.hparams
        d = hp.d_model
        if (hp.get('d_embedding') or d) != d:
            raise NotImplementedError('d_embedding != d_model (input projection) is not on the MI355X path')
        if not hp.get('tie_embedding_weights', True):
            raise NotImplementedError('untied embedding/head weights are not on the MI355X path')
        if hp.get('cross_attention', False):
            raise NotImplementedError('decoder cross-attention (transformer-lm context) is not on the VAE path')
        if d % 64:
            raise ValueError('d_model must be a multiple of 64 (Perceiver heads = d_model // 64, perceiver.py:13)')
        # --- module tree in the reference's registration order (transformer_language_model.py:34-72,
        #     transformer_vae.py:26-40) so state_dict keys and order match
        self.input_layer = nn.Sequential(nn.Embedding(VOCAB_SIZE, d), nn.Dropout(p=hp.get('input_dropout', 0.0)))
        self.context_layer = None
        self.output_layer = nn.Sequential(nn.Linear(d, d), nn.GELU(), nn.LayerNorm(d), nn.Linear(d, VOCAB_SIZE))
        self.output_layer[3].weight = self.input_layer[0].weight
        sparse = hp.get('sparse_self_attention', True)
        self.decoder_layers = nn.ModuleList([
            TransformerLayer(d, hp.num_heads, causal=True, sparse_self_attention=False if not sparse else hp.attn_window_size)
            for _ in range(hp.num_layers)])
        self.example_input_array = None
        self.encoder_input_layer = deepcopy(self.input_layer)
        self.encoder_input_layer[0].weight = self.input_layer[0].weight
        self.q_of_z_given_x = ConditionalGaussian(d, hp.latent_depth)
        self.encoder = Perceiver(num_layers=hp.num_layers // 2, num_latents=64, d_model=d, bottleneck_width=1)
        self.z_projections = nn.ModuleList([nn.Linear(hp.latent_depth, d) for _ in range(hp.num_layers)])
        self._ehp = _EngineHP(hp)
        if device is None:
            device = 'cuda' if torch.cuda.is_available() else 'cpu'
        self._flat = None
        self._engine = None
        self._bind_flat(torch.device(device))
        self._norm_part = None
        self._norm_valid = False
        self._dp = None
        self._log_consts = None
        self.logged_reduced = {}
        self.comm_probe = None     # a list: (start, end) HIP events of each step's exposed all-reduce tail (bench.py)
        self._step_seed = 7295
        # DDP's flag (Lightning sets it through no_sync under accumulate_grad_batches): False marks a gradient-
        # accumulation micro-step that no optimiser step follows -- its backward runs no all-reduce (the final
        # micro-step's buckets carry the accumulated sum) and on_after_backward applies its clip in place
        self.require_backward_grad_sync = True
        self.token_weights = None

    # ------------------------------------------------------------------ flat arena plumbing
    def _bind_flat(self, device):
        old = self._flat
        flat = FlatParams(self._ehp, device)
        with torch.no_grad():
            for name in flat.offsets:
                src = self.get_parameter(name)
                flat.view(name).copy_(src.detach().to(device))
        for name in flat.offsets:
            mod_name, _, pname = name.rpartition('.')
            mod = self.get_submodule(mod_name)
            mod._parameters[pname] = nn.Parameter(flat.view(name), requires_grad=True)
        emb = self.input_layer[0].weight
        self.output_layer[3].weight = emb
        self.encoder_input_layer[0].weight = emb
        self._flat = flat
        self._engine = VAEEngine(self._ehp, flat) if device.type == 'cuda' else None
        self._grads_attached = False
        del old

    def _apply(self, fn, recurse=True):
        probe = fn(torch.zeros(1, device=self._flat.device))
        if probe.dtype != torch.float32:
            raise RuntimeError('TransformerVAE keeps f32 master weights (bf16 copies are internal)')
        if probe.device != self._flat.device:
            self._bind_flat(probe.device)
        return self

    @property
    def device(self):
        return self._flat.device

    def _require_engine(self):
        if self._engine is None:
            raise RuntimeError('TransformerVAE.training_step runs on the MI355X HIP kernels: move the model to a '
                               'GPU (model.cuda()). There is no CPU fallback.')
        return self._engine

    def zero_grad_flat(self):
        self._flat.grad.zero_()
        self._attach_grads()
        self._norm_valid = False

    def zero_grad(self, set_to_none: bool = True):
        self.zero_grad_flat()

    def _attach_grads(self):
        flat = self._flat
        for name in flat.live_names:
            p = self.get_parameter(name)
            p.grad = flat.g(name)
        self._grads_attached = True

    @property
    def _anchor(self):
        return self.q_of_z_given_x.linear.bias

    def _grads_alive(self):
        p = self._anchor
        return self._grads_attached and p.grad is not None and p.grad.data_ptr() == self._flat.g(
            'q_of_z_given_x.linear.bias').data_ptr()

    # ------------------------------------------------------------------ data parallel (RCCL over xGMI)
    def enable_data_parallel(self, group=None, bucket_mb: Optional[float] = None):
        """Pure DP: grads are averaged with bucketed async all-reduces launched while the
        backward is still running (the arena is in gradient-ready order, so buckets are contiguous). A bucket
        closes once >= bucket_mb of gradients are final (default 25 MB, env SVAE_DP_BUCKET_MB): at C2 the first
        all-reduce starts after two decoder layers' backward (12.6 MB each) instead of five at 64 MB."""
        if bucket_mb is None:
            bucket_mb = float(os.environ.get('SVAE_DP_BUCKET_MB', '25'))
        self._dp = {'group': group, 'bucket': int(bucket_mb * 2 ** 20 / 4), 'start': 0, 'works': [],
                    'world': dist.get_world_size(group)}
        # identical initial weights on every rank
        dist.broadcast(self._flat.master, 0, group=group)
        self._flat.shadow_version = -1

    def _dp_ready(self, end, final=False):
        """Called by the engine backward each time the arena prefix [0, end) holds final gradients."""
        dp = self._dp
        if dp is None:
            return
        if end - dp['start'] >= dp['bucket'] or (final and end > dp['start']):
            seg = self._flat.grad[dp['start']:end]
            # the backward ran on loss / world, so a SUM all-reduce leaves the average (no extra pass)
            dp['works'].append(dist.all_reduce(seg, op=dist.ReduceOp.SUM, group=dp['group'], async_op=True))
            dp['start'] = end

    def _dp_finish(self):
        dp = self._dp
        if dp is None:
            return
        probe = self.comm_probe
        if probe is not None:
            # exposed communication: from the end of the backward on the compute stream (every bucket but the last
            # already in flight) to the point where that stream may proceed past the last bucket's all-reduce
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
        self._dp_ready(self._flat.n_live, final=True)
        for w in dp['works']:
            w.wait()
        if probe is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            probe.append((e0, e1))
        dp['works'] = []
        dp['start'] = 0

    # ------------------------------------------------------------------ training step
    def _batch_inputs(self, batch):
        ids = batch['token_ids']
        pad = getattr(ids, 'padding', None)
        if isinstance(ids, PaddedTensor):
            ids = ids.as_raw()
        dev = self.device
        ids = ids.to(dev, non_blocking=True)
        if pad is not None:
            pad = pad.to(dev, non_blocking=True)
            if pad.shape != ids.shape:
                pad = None
        ntok = batch['num_tokens'].to(dev, non_blocking=True)
        return ids, pad, ntok

    def training_step(self, batch: Dict[str, Any], batch_index: int = 0, stage: str = 'train', eps=None,
                      dropout: Optional[float] = None, eps_marginal=None):
        """transformer_vae.py:42-66. `eps` (injected N(0,1) noise [B,1,latent]), `eps_marginal` (the 10
        marginal_kl draws [10,B,1,latent]) and `dropout` override the in-kernel noise / the nn.Dropout(0.1) rate
        for parity runs."""
        eng = self._require_engine()
        ids, pad, ntok = self._batch_inputs(batch)
        train = stage == 'train' and self.training
        p = (0.1 if train else 0.0) if dropout is None else dropout
        self._step_seed += 1
        kw = float(self.hparams.kl_weight)
        out = eng.forward(ids, ntok, pad=pad if pad is not None else False, eps=eps, seed=self._step_seed,
                          kl_weight=kw, dropout=p)
        self._last = out
        self._kl_weight_used = kw
        self.log(stage + '_kl', out['train_kl'])                       # continuous_autoencoder.py:50
        self.log(stage + '_nll', out['nll'])                           # language_model.py:112
        mu, logvar = out['mu'].view(-1, 1, self.hparams.latent_depth), out['logvar'].view(-1, 1, self.hparams.latent_depth)
        scale = logvar.exp().sqrt()
        if ids.shape[0] > 1 and self.hparams.get('log_mutual_info', True):
            # transformer_vae.py:59-61: kl - marginal_kl(posterior), fused (engine.mutual_info)
            self.log(stage + '_mc_mutual_info', eng.mutual_info(out, eps=eps_marginal))
        else:
            # not logged for this batch: drop an earlier step's value so it is neither reported nor reduced again
            self.logged.pop(stage + '_mc_mutual_info', None)
        if stage == 'train':
            loss = _StepFn.apply(self._anchor, self, out['loss'])
            # (validate_args=False: the argument check reads the scale back to the host, a sync per step)
            return {'loss': loss, 'posterior': Normal(loc=mu.detach(), scale=scale.detach(), validate_args=False)}
        if stage == 'val':
            self.log('val_loss', out['nll'] + out['kl'])
            if self.token_weights is not None:
                # language_model.py:106-110: robust_cross_entropy(weight=token_weights) * bytes_per_token / log 2;
                # bytes_per_token is [B] there, logged here as its batch mean
                bpt = batch['num_bytes'].to(self.device, torch.float32) / ntok.to(torch.float32)
                tw = self.token_weights.to(self.device, torch.float32).contiguous()
                self.log('val_bpb', (eng.weighted_nll(tw) * bpt).mean() / math.log(2))
        return None

    def validation_step(self, batch, batch_index: int = 0):
        with torch.no_grad():
            was = self.training
            self.eval()
            try:
                return self.training_step(batch, batch_index, stage='val')
            finally:
                self.train(was)

    def _run_backward(self, gloss):
        eng = self._require_engine()
        if not self._grads_alive():
            self.zero_grad_flat()
        g = gloss.reshape(()).to(torch.float32)
        if self._dp is not None:
            g = g / self._dp['world']
        # all-reduce only on the micro-step an optimiser step follows (DDP no_sync semantics): the buckets then
        # reduce the accumulated sum once; reducing every micro-step would add the already-averaged earlier
        # micro-gradients world times over
        sync = self._dp is not None and self.require_backward_grad_sync
        eng.backward(g, self._kl_weight_used, ready=self._dp_ready if sync else None)
        if sync:
            self._dp_finish()
        self._norm_valid = False

    def _norm_partials(self, fresh=True):
        if self._norm_part is None:
            self._norm_part = torch.empty(1024, device=self.device)
        if fresh or not self._norm_valid:
            K.sumsq(self._flat.grad, self._flat.n_live, self._norm_part)
            self._norm_valid = True
        return self._norm_part

    def grad_norm(self):
        return self._norm_partials(fresh=True).sum().sqrt()

    def _local_grad_scale(self):
        """Factor from the arena's contents to the gradient the reference would clip here. Under data parallelism
        the backward ran on loss / world, so an accumulation micro-step (no all-reduce yet) leaves G_local / world
        in the arena, while DDP's no_sync micro-step clips the unscaled local G. After the all-reduce the arena
        holds the rank mean, which is what DDP clips."""
        if self._dp is not None and not self.require_backward_grad_sync:
            return float(self._dp['world'])
        return 1.0

    def on_after_backward(self):
        """language_model.py:120-122 (clip_grad_norm_ + `grad_norm` log) and continuous_autoencoder.py:28-39."""
        scale = self._local_grad_scale()
        norm = self.grad_norm()
        self.log('grad_norm', norm * scale if scale != 1.0 else norm)
        if not self.require_backward_grad_sync:
            # an accumulation micro-step: the reference clips after every backward (language_model.py:120-122),
            # so this partial gradient is clipped now; the last micro-step's clip is fused into RAdam. The arena
            # holds G / scale: clipping it at threshold / scale is clipping G at the threshold
            K.clip_grad(self._flat.grad, self._flat.n_live, self._norm_partials(fresh=False),
                        float(self.hparams.get('grad_clip_threshold', 5.0)) / scale)
            self._norm_valid = False
        self.anneal_kl()                   # continuous_autoencoder.py:28-39

    LOGGED_REDUCE_KEYS = ('loss', 'train_nll', 'train_kl', 'train_mc_mutual_info', 'grad_norm')

    def reduce_logged(self, keys=LOGGED_REDUCE_KEYS):
        """the logged scalars averaged over the data-parallel ranks for reporting (each rank's
        training step logs its local values, language_model.py:112, continuous_autoencoder.py:50,
        transformer_vae.py:61). One all-reduce of a FIXED-length vector: for every key of `keys`, the value (0 where
        this rank did not log it) and a presence count, so ranks whose batches log different key sets (a
        1-sequence token-budget batch logs no `train_mc_mutual_info`) still issue identical collectives; a key
        is the mean over the ranks that logged it, and is dropped where no rank did. Everything stays on the
        device: the vector is stacked from device scalars (no host-to-device copy), `wait()` on RCCL only orders
        the caller's stream after the collective, and the means and presence counts land in `logged_reduced`
        (device tensors). `logged_values()` reads them back to the host -- the trainer calls it only where it
        prints a log line (rank 0, every log_every_n_steps), so an optimiser step carries no host synchronisation.
        Every rank calls it at the same optimiser steps (the trainer does, once per optimiser step)."""
        dp = self._dp
        if dp is None:
            return
        keys = tuple(keys)
        if self._log_consts is None or self._log_consts[0].device != self._flat.master.device:
            dev = self._flat.master.device
            self._log_consts = (torch.zeros((), dtype=torch.float32, device=dev),
                                torch.ones((), dtype=torch.float32, device=dev))
        zero, one = self._log_consts
        present = [k in self.logged for k in keys]
        vals = torch.stack([torch.as_tensor(self.logged[k], dtype=torch.float32, device=zero.device).reshape(())
                            if p else zero for k, p in zip(keys, present)]
                           + [one if p else zero for p in present])
        dist.all_reduce(vals, op=dist.ReduceOp.SUM, group=dp['group'], async_op=True).wait()
        n = len(keys)
        means = vals[:n] / vals[n:].clamp_min(1.0)
        self.logged_reduced = {k: (means[i], vals[n + i]) for i, k in enumerate(keys)}

    def logged_values(self):
        """Host values of the logged scalars: the data-parallel means of `reduce_logged` where a reduction ran
        (a key no rank logged is dropped: its presence count is read here), the local values otherwise. One
        host synchronisation (one stacked transfer); call it only where the values are printed. Warns when the
        last step's P-head recomputed saturated rows (a logit > 88 nats above the label's: a diverging run, whose
        exact fix-up costs ~0.3 ms per row)."""
        local = {k: v for k, v in self.logged.items() if k not in self.logged_reduced}
        dev_keys, dev_vals, out = [], [], {}
        for k, v in local.items():
            if torch.is_tensor(v):
                dev_keys.append(k)
                dev_vals.append(v.detach().reshape(()).float())
            else:
                out[k] = v
        red = list(self.logged_reduced.items())
        last = getattr(self, '_last', None)
        sat = last.get('ce_saturated') if isinstance(last, dict) else None
        flat = dev_vals + [m.reshape(()).float() for _, (m, _) in red] + [c.reshape(()).float() for _, (_, c) in red]
        if sat is not None:
            flat.append(sat.reshape(()).float())
        host = torch.stack(flat).tolist() if flat else []
        for i, k in enumerate(dev_keys):
            out[k] = host[i]
        n0, n = len(dev_keys), len(red)
        for i, (k, _) in enumerate(red):
            if host[n0 + n + i] > 0:
                out[k] = host[n0 + i]
        if sat is not None and host[-1] > 0:
            warnings.warn(f'{int(host[-1])} token rows of the last step saturated the P-head (a logit > 88 nats above '
                          'the label logit) and were recomputed exactly: the run may be diverging', RuntimeWarning)
        return out

    # ------------------------------------------------------------------ inference-side helpers
    @torch.no_grad()
    def reconstruct(self, x, z, precision: str = 'bf16'):
        """transformer_vae.py:85-93 on the device (no autograd): x = input_layer(ids) [B, L, d] f32 (a
        PaddedTensor carrying the padding mask, or plain), z [B, 1, latent] -> logits [B, L, V]: bf16 from the
        training kernels, or f32 from the fp32 kernel mode (precision='fp32', the argmax-parity mode)."""
        eng = self._require_engine()
        pad = getattr(x, 'padding', None)
        x = x.as_raw() if isinstance(x, PaddedTensor) else x
        x = x.float().contiguous()
        z = z.reshape(z.shape[0], -1).float().contiguous()
        if precision == 'fp32':
            return eng.reconstruct_f32(x, z, pad)
        return eng.reconstruct(x, z, pad)

    @torch.no_grad()
    def p_of_x_given_z(self, x, z, labels, padding=None):
        """continuous_autoencoder.py:82-88: log p(x|z) summed over the sequence, for x = input_layer(ids)
        [..., L, d] (a PaddedTensor or plain; `padding` overrides its mask), z [..., 1, latent], labels
        [..., L-1]. Returns [...]. Decoder + vocabulary head run in the HIP kernels; the head keeps only its CE
        statistics (the [.., L, V] logits are never stored)."""
        eng = self._require_engine()
        pad = padding if padding is not None else getattr(x, 'padding', None)
        x = x.as_raw() if isinstance(x, PaddedTensor) else x
        lead, L, d = x.shape[:-2], x.shape[-2], x.shape[-1]
        Z = z.shape[-1]
        if len(lead) == 1:
            x4, z3, l3 = x.unsqueeze(0), z.reshape(1, lead[0], Z), labels.reshape(1, lead[0], L - 1)
        else:
            G = 1
            for n in lead[:-1]:
                G *= n
            # merge the leading dims without materialising an expanded x (view when possible)
            x4 = x.reshape(G, lead[-1], L, d) if x.is_contiguous() else x.flatten(0, len(lead) - 2)
            z3, l3 = z.reshape(G, lead[-1], Z), labels.reshape(G, lead[-1], L - 1)
        p3 = pad.expand(*lead, L).reshape(x4.shape[0], x4.shape[1], L) if pad is not None else None
        return eng.seq_log_prob(x4, l3, z3.float(), p3).reshape(lead)

    @torch.no_grad()
    def test_step(self, batch: Dict[str, Any], batch_index: int = 0):
        """transformer_vae.py:71-79: importance-weighted NLL with 100 posterior samples (100 chunks of 1)."""
        eng = self._require_engine()
        ids, pad, ntok = self._batch_inputs(batch)
        Z = self.hparams.latent_depth
        stats = eng.posterior(ids, pad if pad is not None else False)
        mu = stats[:, :Z].reshape(-1, 1, Z).clone()
        posterior = Normal(mu, stats[:, Z:].exp().sqrt().reshape(-1, 1, Z))
        x = self.embed(PaddedTensor.from_raw(ids, pad) if pad is not None else ids)
        log_prob = self.estimate_log_prob_iw(posterior, x, ids.long(), num_samples=100, num_iter=100) / ntok
        nll_iw = -log_prob.mean()
        self.log('nll_iw', nll_iw, on_step=True)
        return nll_iw

    @torch.no_grad()
    def sample(self, max_length: int, batch_size: int = 1, **kwargs):
        """transformer_vae.py:95-128: autoregressive decoding with a KV cache (f32 kernels, one HIP graph per
        step). kwargs: z [B, 1, latent] (default N(0, I)), and GenerationState's top_k / top_p / temperature /
        repetition_penalty; use_graph=False steps eagerly. Returns output_ids[:, 1:] (None below kl_weight 1,
        as in the reference)."""
        if self.hparams.kl_weight < 1.0:
            return None
        eng = self._require_engine()
        z = kwargs.pop('z', None)
        use_graph = kwargs.pop('use_graph', True)
        if z is None:
            z = torch.randn(batch_size, 1, self.hparams.latent_depth, device=self.device)
        start = self.start_token if self.start_token is not None else 1      # [CLS] (text_data_module.py:271)
        end = self.end_token if self.end_token is not None else 2            # [SEP]
        state = GenerationState(max_length, batch_size, start, end, device=self.device, **kwargs)
        return KVDecoder(eng, state, z.to(self.device), use_graph=use_graph).run()

    @torch.no_grad()
    def embed(self, ids):
        """input_layer(ids) as a PaddedTensor (the reference's x, transformer_vae.py:45)."""
        pad = getattr(ids, 'padding', None)
        raw = ids.as_raw() if isinstance(ids, PaddedTensor) else ids
        raw = raw.to(self.device)
        B, L = raw.shape
        ids32 = raw.to(torch.int32).contiguous()
        out = torch.empty(B, L, self.hparams.d_model, device=self.device)
        K.embedding_fwd(ids32, self._flat.f('input_layer.0.weight'), out, B * L, self.hparams.d_model)
        return PaddedTensor.from_raw(out, pad.to(self.device)) if pad is not None else out

    @torch.no_grad()
    def predict(self, batch, batch_idx: int = 0, dataloader_idx: Optional[int] = None):
        """transformer_vae.py:81-83: q(z|x) for a batch."""
        self.training_step(batch, stage='predict', dropout=0.0)
        mu, logvar = self._last['mu'], self._last['logvar']
        return Normal(mu.view(-1, 1, mu.shape[-1]).clone(), logvar.exp().sqrt().view(-1, 1, mu.shape[-1]))
