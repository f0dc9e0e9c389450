"""The TransformerVAE training step on MI355X: explicit forward / backward over libsvae kernels.

Reference path (norabelrose/sparse-vae): `TransformerVAE.training_step` (transformer_vae.py:42-66) with the
Perceiver encoder (perceiver.py:39-50), `sample_z` (continuous_autoencoder.py:42-52), `reconstruct`
(transformer_vae.py:85-93), the tied output head (transformer_language_model.py:55-63) and
`robust_cross_entropy` (language_model.py:161-170), differentiated by autograd.

Here the step is one explicit pass each way. Parameters live in one flat f32 arena (master weights) with a
bf16 shadow (GEMM operands) and one flat f32 gradient arena, laid out in gradient-ready order so that
data-parallel buckets are contiguous ranges. Activations stay resident in HBM between the passes (no
recomputation: 288 GB per GPU makes activation checkpointing unnecessary at these sizes).

Numerics: GEMM/attention operands bf16 with f32 accumulation; residual stream, LayerNorm statistics,
mu/logvar, KL, softmax statistics and all gradients of the residual stream in f32.
"""
import math
import os
from collections import OrderedDict

import torch

from . import kernels as K
from ._native import COLSUM_MAX, LN_MULTI_MAX, ZPROJ_MAX
from ._native import EPI_BF16, EPI_F32, EPI_F32_ACC, EPI_GELU, EPI_GELU_BWD, EPI_DROPOUT_RESID, \
    EPI_ROTARY_BF16, EPI_CE_STATS, EPI_F32_ATOMIC, EPI_CE_PROB, EPI_ROWSCALE_GATHER

bf16, f32 = torch.bfloat16, torch.float32
ALIGN = 64
CE_CHUNK_NUMEL = 2 ** 30      # language_model.py:163


# ---------------------------------------------------------------------------------------- layout
def _attn_entries(pre, d, learned):
    out = []
    if learned:
        out.append((pre + 'learned_queries', (1, learned, d)))
        names = ['k_linear', 'v_linear']
    else:
        names = ['q_linear', 'k_linear', 'v_linear']
    out += [(pre + n + '.weight', (d, d)) for n in names]      # adjacent -> one [n*d, d] GEMM operand
    out += [(pre + n + '.bias', (d,)) for n in names]           # adjacent -> one bias vector
    out += [(pre + 'output_linear.weight', (d, d)), (pre + 'output_linear.bias', (d,))]
    return out


def _ctx_ln_entries(pre, d):
    return [(pre + 'context_layer_norm.weight', (d,)), (pre + 'context_layer_norm.bias', (d,))]


def _layer_entries(pre, d, learned=None, cross=False, ctx_ln=True):
    """ctx_ln=False: the cross-attention layer's context LayerNorm is laid out elsewhere (layout_entries: after every
    middle layer, where the batched context-LayerNorm backward completes it)."""
    out = _attn_entries(pre + 'attention.', d, learned)
    out += [(pre + 'attn_layer_norm.weight', (d,)), (pre + 'attn_layer_norm.bias', (d,))]
    if cross:
        out += _attn_entries(pre + 'cross_attention.', d, None)
        out += [(pre + 'cross_attn_layer_norm.weight', (d,)), (pre + 'cross_attn_layer_norm.bias', (d,))]
        if ctx_ln:
            out += _ctx_ln_entries(pre, d)
    out += [(pre + 'ffn.0.weight', (4 * d, d)), (pre + 'ffn.0.bias', (4 * d,)), (pre + 'ffn.2.weight', (d, 4 * d)),
            (pre + 'ffn_layer_norm.weight', (d,)), (pre + 'ffn_layer_norm.bias', (d,))]
    return out


def _pos_linear_entries(pre, d):
    return [(pre + 'pos_linear.weight', (d, d)), (pre + 'pos_linear.bias', (d,))]


def ctx_ln_batched(hp):
    """The encoder middle layers' context LayerNorms -- one per middle layer, all over the same x_emb
    (transformer_layer.py:52, perceiver.py:43-46) -- run as batched passes: one forward pass writes every layer's
    normalised context (svae_layernorm_fwd_multi) and one backward pass after the middle layers' backward sums their
    gradients (svae_layernorm_bwd_multi), instead of one forward and one backward pass per layer. On with >= 2 middle
    layers (C4 / C5: 4); SVAE_CTX_LN_BATCH=0 restores the per-layer passes (A/B runs)."""
    return hp.enc_layers - 2 >= 2 and os.environ.get('SVAE_CTX_LN_BATCH', '1') != '0'


def layout_entries(hp):
    """(name, shape) in gradient-ready order (head -> decoder L-1..0 -> q(z|x) -> encoder -> embedding),
    then the parameters that never receive a gradient (Attention.pos_linear, attention.py:39)."""
    d, V, Z, N = hp.d_model, hp.vocab_size, hp.latent_depth, hp.num_latents
    live = [('output_layer.0.weight', (d, d)), ('output_layer.0.bias', (d,)),
            ('output_layer.2.weight', (d,)), ('output_layer.2.bias', (d,)), ('output_layer.3.bias', (V,))]
    dead = []
    for i in reversed(range(hp.num_layers)):
        live += _layer_entries(f'decoder_layers.{i}.', d)
        live += [(f'z_projections.{i}.weight', (d, Z)), (f'z_projections.{i}.bias', (d,))]
        dead += _pos_linear_entries(f'decoder_layers.{i}.attention.', d)
    live += [('q_of_z_given_x.linear.weight', (2 * Z, d)), ('q_of_z_given_x.linear.bias', (2 * Z,))]
    live += _layer_entries('encoder.bottleneck.', d, learned=1)
    dead += _pos_linear_entries('encoder.bottleneck.attention.', d)
    nmid = hp.enc_layers - 2
    batched = ctx_ln_batched(hp)
    for j in reversed(range(nmid)):
        live += _layer_entries(f'encoder.middle_layers.{j}.', d, cross=True, ctx_ln=not batched)
        dead += _pos_linear_entries(f'encoder.middle_layers.{j}.attention.', d)
        dead += _pos_linear_entries(f'encoder.middle_layers.{j}.cross_attention.', d)
    if batched:   # (their gradients complete together, after the middle layers' backward)
        for j in reversed(range(nmid)):
            live += _ctx_ln_entries(f'encoder.middle_layers.{j}.', d)
    live += _layer_entries('encoder.first_layer.', d, learned=N)
    dead += _pos_linear_entries('encoder.first_layer.attention.', d)
    live += [('input_layer.0.weight', (V, d))]
    return live, dead


class FlatParams:
    """f32 master arena + bf16 shadow + f32 grad arena; `views[name]` etc. are shaped views."""

    def __init__(self, hp, device):
        live, dead = layout_entries(hp)
        # the layout's choice for the context LayerNorms (the engine follows it, whatever the environment says later)
        self.ctx_batched = ctx_ln_batched(hp)
        self.offsets = OrderedDict()
        off = 0
        for name, shape in live + dead:
            n = math.prod(shape)
            self.offsets[name] = (off, shape)
            off += -(-n // ALIGN) * ALIGN
            if name == live[-1][0]:
                self.n_live = off
        self.total = off
        self.live_names = [n for n, _ in live]
        self.device = torch.device(device)
        self.master = torch.zeros(self.total, dtype=f32, device=self.device)
        self.shadow = torch.zeros(self.total, dtype=bf16, device=self.device) if self.device.type == 'cuda' else None
        # transposed bf16 copies of the weight blocks the dX GEMMs read (K-contiguous B operand), same offsets
        self.shadow_t = torch.zeros_like(self.shadow) if self.shadow is not None else None
        self.t_blocks = OrderedDict()          # (name, rows, cols) -> (offset, rows, cols)
        self._t_table = None
        self.grad = torch.zeros(self.total, dtype=f32, device=self.device)
        self.shadow_version = -1

    def end(self, name):
        off, shape = self.offsets[name]
        return off + -(-math.prod(shape) // ALIGN) * ALIGN

    def view(self, name, buf=None):
        off, shape = self.offsets[name]
        buf = self.master if buf is None else buf
        return buf[off:off + math.prod(shape)].view(shape)

    def w(self, name):      # bf16 GEMM operand
        return self.view(name, self.shadow)

    def f(self, name):      # f32 master (biases, LayerNorm affine)
        return self.view(name)

    def g(self, name):
        return self.view(name, self.grad)

    def wT(self, name, rows, cols):
        """bf16 W^T [cols][rows] of the rows x cols weight block starting at `name` (e.g. a fused q|k|v
        block), kept in sync with the shadow; the dX GEMM's K-contiguous B operand."""
        key = (name, rows, cols)
        off = self.offsets[name][0]
        if key not in self.t_blocks:
            assert rows % 8 == 0 and cols % 8 == 0, key
            for o, r, c in self.t_blocks.values():
                assert off + rows * cols <= o or o + r * c <= off, f'overlapping transposed blocks at {name}'
            self.t_blocks[key] = (off, rows, cols)
            self._t_table = None
            self.refresh_transposed([key])
        return self.shadow_t[off:off + rows * cols].view(cols, rows)

    def refresh_transposed(self, keys=None):
        """Re-derive the transposed shadows from the shadow (after every shadow write)."""
        if not self.t_blocks:
            return
        if keys is None and self._t_table is not None:
            table, nb, tiles = self._t_table
        else:
            rows_tab, tiles = [], 0
            for k in (keys if keys is not None else self.t_blocks):
                o, r, c = self.t_blocks[k]
                rows_tab.append([o, r, c, tiles])
                tiles += -(-r // 64) * -(-c // 64)
            table = torch.tensor(rows_tab, dtype=torch.int64).to(self.device)
            nb = len(rows_tab)
            if keys is None:
                self._t_table = (table, nb, tiles)
        K.transpose_blocks(self.shadow, self.shadow_t, table, nb, tiles)

    def sync_shadow(self, force=False):
        """Refresh the bf16 shadow if the master changed outside the fused optimiser (load_state_dict,
        initialize_weights, manual edits) — detected through the arena's shared version counter."""
        if force or self.master._version != self.shadow_version:
            K.cast_bf16(self.master, self.shadow)
            self.refresh_transposed()
            self.shadow_version = self.master._version


# ---------------------------------------------------------------------------------------- workspace
class Workspace:
    """Named device buffers reused across steps. A buffer still being read by the weight-gradient stream is
    fenced: get() makes the caller's stream wait for that read before handing the buffer out again."""

    def __init__(self, device):
        self.device = device
        self.bufs = {}
        self.busy = {}      # storage data_ptr -> event recorded after the last side-stream read

    def fence(self, t):
        ev = self.busy.pop(t.untyped_storage().data_ptr(), None)
        if ev is not None:
            torch.cuda.current_stream().wait_event(ev)

    def get(self, name, shape, dtype=bf16, zero=False):
        t = self.bufs.get(name)
        if t is None or t.shape != torch.Size(shape) or t.dtype != dtype:
            t = torch.empty(shape, dtype=dtype, device=self.device)
            self.bufs[name] = t
        if self.busy:
            self.fence(t)
        if zero:
            t.zero_()
        return t


def rotary_table(positions, d, max_pos=10000):
    """cos/sin table exactly as encode_position_rotary builds it (attention.py:194-200), in fp32 on the
    host so the factors are bitwise those of the fp32 reference; layout [pos][d/2][2]. max_pos is 10000 for
    dense attention and 2 * window * 32 for SparseAttention (attention.py:52)."""
    half = d // 2
    freqs = torch.arange(half, dtype=f32)
    pos = torch.arange(0, positions, dtype=f32)
    theta = max_pos ** (-freqs / half)
    ang = pos[:, None] * theta
    return torch.stack([ang.cos(), ang.sin()], dim=-1).contiguous()


def _mix_seed(a, b):
    x = (a * 0x9E3779B97F4A7C15 + b * 0xBF58476D1CE4E5B9 + 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    x ^= x >> 31
    return x


# ---------------------------------------------------------------------------------------- engine
class VAEEngine:
    def __init__(self, hp, flat: FlatParams):
        self.hp = hp
        self.P = flat
        self.ws = Workspace(flat.device)
        self.d = hp.d_model
        self.H = hp.num_heads
        self.He = hp.d_model // 64
        assert self.d % self.H == 0 and self.d % 64 == 0
        self.hd = self.d // self.H
        self._rot = {}
        self.window = getattr(hp, 'attn_window', 0)     # decoder self-attention: 0 dense, > 0 sliding window
        self.saved = None
        self.probe = None      # list -> HIP events around each vocab-head GEMM launch (bench roofline)
        # SVAE_DW_STREAM=1: weight-gradient GEMMs on a second stream, off the dX critical path of the backward
        # (they feed nothing else in it). Measured at C2: 15.33 vs 15.37 ms/step -- the overlap is eaten by
        # contention (LayerNorm backward 35 -> 85 us beside a GEMM, the head dW doubled beside the head dX), so
        # the default keeps one stream.
        # vocabulary head + cross entropy of the training step: 'prob' stores P = exp(logit - label logit) and runs
        # the backward on it without a dlogits pass (svae.h, P-head); 'logits' stores the bf16 logits and rewrites
        # them into dlogits in place (ce_grad) -- the round-1 path, kept for A/B runs (SVAE_HEAD=logits)
        self.head_mode = os.environ.get('SVAE_HEAD', 'prob')
        assert self.head_mode in ('prob', 'logits'), self.head_mode
        # the two dW GEMMs of the FFN, and the attention output projection's with the Q/K/V projection's, run as one
        # paired launch each (kernels.linear_dw_pair); SVAE_DW_PAIR=0 launches them one by one (A/B runs)
        self.dw_pair = os.environ.get('SVAE_DW_PAIR', '1') != '0'
        # decoder residual adds in a separate fused residual + dropout + LayerNorm pass (layer_fwd's fuse, SVAE_FUSE_LN=1)
        # instead of the projections' f32 residual epilogues + LayerNorm passes. Off by default: measured at C2 it moves
        # 36 B per element and layer against 28 (the projection output makes an f32 round trip), +0.125 ms of kernel
        # time per step (profiles/r03f_*); at C4 +0.5-0.8 ms/step
        self.fuse_ln = os.environ.get('SVAE_FUSE_LN', '0') != '0'
        # attention backward delta = rowsum(dO . O): SVAE_DELTA_FUSED=1 has the dO GEMM's epilogue write it (built and
        # tested, measured no faster: C2 12.725 / 12.696 vs 12.648 / 12.681 ms, C4 neutral,
        # profiles/r04j_delta_ab.log); default: the attention backward's own delta pass
        self.delta_fused = os.environ.get('SVAE_DELTA_FUSED', '0') != '0'
        # the attention forward's copy of O for the backward's delta: the bf16 residual O - bf16(O) (2 B per element)
        # unless SVAE_ATTN_O32=1 (the f32 copy, 4 B; A/B runs)
        self.o32_mode = os.environ.get('SVAE_ATTN_O32', '0') != '0'
        # the last decoder layer's dropout + residual GEMM epilogue also writes the bf16 copy of its output (the vocab
        # head's input) instead of a separate [T, d] cast pass; SVAE_RESID_BF16=0 restores the cast (A/B runs)
        self.resid_bf16 = os.environ.get('SVAE_RESID_BF16', '1') != '0'
        # and the head's d x GEMM writes the top decoder layer's dropout-masked bf16 gradient (SVAE_HEAD_G2=0: the
        # layer backward's own dropout_bwd_cast pass)
        self.head_g2 = os.environ.get('SVAE_HEAD_G2', '1') != '0'
        # the head LayerNorm's backward writes bf16(dx * GELU') directly (SVAE_LN_GELU=0: f32 dx + a gelu_bwd pass)
        self.ln_gelu = os.environ.get('SVAE_LN_GELU', '1') != '0'
        # the step's token inputs (ids32, labels, padding mask, token counts) and its scalars (loss, gradient scales)
        # in one launch each instead of torch's copy / fill / mul / add ops (SVAE_SMALL_FUSED=0: the torch ops)
        self.small_fused = os.environ.get('SVAE_SMALL_FUSED', '1') != '0'
        # the decoder layers' z-projection backwards in one launch (SVAE_ZPROJ_BATCH=0: one launch per layer)
        self.zp_batch = os.environ.get('SVAE_ZPROJ_BATCH', '1') != '0'
        # and their forwards (one launch; each layer's first LayerNorm splices its rows in; SVAE_ZPROJ_FWD_BATCH=0: a
        # skinny GEMM per layer into the position-0 rows)
        self.zf_batch = os.environ.get('SVAE_ZPROJ_FWD_BATCH', '1') != '0'
        self._zp_pending, self._zp_ctx = [], None
        # the LayerNorm-affine gradient partials of consecutive LayerNorm backwards summed in one launch
        # (SVAE_COLSUM_BATCH=0: one colsum launch per LayerNorm, for A/B runs)
        self.cs_batch = os.environ.get('SVAE_COLSUM_BATCH', '1') != '0'
        self._cs_pending = []
        self.ncu = (torch.cuda.get_device_properties(flat.device).multi_processor_count
                    if flat.device.type == 'cuda' else 256)
        self.side = None
        if flat.device.type == 'cuda' and os.environ.get('SVAE_DW_STREAM', '0') != '0':
            self.side = torch.cuda.Stream(device=flat.device)

    # ------------------------------------------------------------------ helpers
    def rot(self, L, window=0):
        """Rotary cos/sin table for positions < L; window > 0 selects SparseAttention's base 2 * window * 32."""
        need = max(L, self.hp.num_latents)
        base = 2 * window * 32 if window else 10000
        t = self._rot.get(base)
        if t is None or t.shape[0] < need:
            t = rotary_table(max(need, 512), self.d, base).to(self.P.device)
            self._rot[base] = t
        return t

    def _ln_fwd(self, name, x, rows, tag, zsplice=None):
        """zsplice = (zrows f32 [rows / zmod, D], zmod): rows r % zmod == 0 of x are replaced by zrows first."""
        D = self.d
        y = self.ws.get(tag + '.y', (rows, D))
        mean = self.ws.get(tag + '.mean', (rows,), f32)
        rstd = self.ws.get(tag + '.rstd', (rows,), f32)
        if zsplice is not None:
            K.layernorm_fwd_z(x, zsplice[0], zsplice[1], self.P.f(name + '.weight'), self.P.f(name + '.bias'), y, mean,
                              rstd, rows, D)
        else:
            K.layernorm_fwd(x, self.P.f(name + '.weight'), self.P.f(name + '.bias'), y, mean, rstd, rows, D)
        return y, (x, mean, rstd)

    def _ln_bwd(self, name, dy, st, rows, dres, dx, dx_bf=None, bf_drop=None, zsplice=None, gelu=None):
        """LayerNorm backward; gelu = the saved GELU' (bf16) of the linear before the LayerNorm: then only
        dx_bf = bf16(dx * gelu) is written (svae_layernorm_bwd_gelu; dres, dx, bf_drop and zsplice unused)."""
        x, mean, rstd = st
        D = self.d
        wg = self.P.grad[self.P.offsets[name + '.weight'][0]:][:2 * D]   # [weight | bias] grads (adjacent)
        if not self.cs_batch:
            part = self.ws.get('ln.part', (1024 * 2 * D,), f32)
            if gelu is not None:
                K.layernorm_bwd_gelu(dy, x, self.P.f(name + '.weight'), mean, rstd, gelu, dx_bf, wg, rows, D, part)
                return
            K.layernorm_bwd(dy, x, self.P.f(name + '.weight'), mean, rstd, dres, dx, dx_bf, wg, rows, D, part,
                            bf_drop=bf_drop, zsplice=zsplice)
            return
        # the affine-gradient partials wait in their own slice of the workspace; flush_colsum sums up to
        # COLSUM_MAX of them in one launch (at every ready() point and at the end of the backward)
        if len(self._cs_pending) == COLSUM_MAX:
            self.flush_colsum()
        k, n1 = len(self._cs_pending), 1024 * 2 * D
        part = self.ws.get('ln.parts', (COLSUM_MAX * n1,), f32)[k * n1:(k + 1) * n1]
        if gelu is not None:
            K.layernorm_bwd_gelu(dy, x, self.P.f(name + '.weight'), mean, rstd, gelu, dx_bf, wg, rows, D, part,
                                 defer=self._cs_pending)
            return
        K.layernorm_bwd(dy, x, self.P.f(name + '.weight'), mean, rstd, dres, dx, dx_bf, wg, rows, D, part,
                        bf_drop=bf_drop, zsplice=zsplice, defer=self._cs_pending)

    def flush_zproj(self):
        """The deferred z-projection backwards (one svae_zproj_bwd_multi launch, in deferral order)."""
        if self._zp_pending:
            z_bf, dz, B, d, Z = self._zp_ctx
            K.zproj_bwd_multi(self._zp_pending, z_bf, dz, B, d, Z)
            self._zp_pending = []

    def flush_colsum(self):
        """Sum the deferred LayerNorm-affine gradient partials (one svae_colsum_multi launch)."""
        if self._cs_pending:
            K.colsum_multi(self._cs_pending)
            self._cs_pending = []

    def _dw(self, dY, X, wname, rows, n_out, n_in, ldy=None, ldx=None, bias=None, on_side=True):
        bg = None
        if bias is not None:
            off = self.P.offsets[bias][0]
            bg = self.P.grad[off:off + n_out]
        side = self.side if on_side else None
        if side is None:
            K.linear_dw(dY, X, self.P.g(wname), rows, n_out, n_in, ldy, ldx, bgrad=bg)
            return
        side.wait_stream(torch.cuda.current_stream())       # dY (and X) are written
        with torch.cuda.stream(side):
            K.linear_dw(dY, X, self.P.g(wname), rows, n_out, n_in, ldy, ldx, bgrad=bg)
        ev = torch.cuda.Event()
        ev.record(side)
        self.ws.busy[dY.untyped_storage().data_ptr()] = ev   # the next writer of dY's buffer waits for this read

    def _head_dw_splits(self, V, d):
        """Split-K factor of the vocabulary head's dW (M = V, N = d, K = T): 2 when one split leaves the last wave of
        256 x 256 tiles partly empty (C4 / C5: 128 x 3 = 384 tiles on 256 CUs run 1.5 waves; two splits, 768 tiles,
        run 3 full ones: `profiles/r04_head_dw_probe_c4.log`), else 1 (C2: 256 tiles). SVAE_HEAD_DW_SPLITS > 0 forces it."""
        env = int(os.environ.get('SVAE_HEAD_DW_SPLITS', '0') or 0)   # (0: chosen here)
        if env > 0:
            return env
        tiles = -(-V // 256) * -(-d // 256)
        ncu = self.ncu
        eff = lambda s: tiles * s / (ncu * -(-(tiles * s) // ncu))   # noqa: E731
        return 2 if tiles >= ncu and eff(2) > eff(1) + 0.1 else 1

    def _dw_pair(self, j0, j1):
        """Two _dw's ((dY, X, wname, rows, n_out, n_in[, ldy, ldx, bias])) in one paired launch (svae_gemm_pair):
        half the split-K slab traffic of two separate launches. SVAE_DW_PAIR=0 (or the side stream) runs them apart."""
        if self.side is not None or not self.dw_pair:
            for j in (j0, j1):
                self._dw(*j[:6], *(tuple(j[6:]) + (None,) * (9 - len(j))))
            return
        args = []
        for j in (j0, j1):
            dY, X, wname, rows, n_out, n_in = j[:6]
            ldy, ldx, bias = tuple(j[6:]) + (None,) * (9 - len(j))
            bg = None
            if bias is not None:
                off = self.P.offsets[bias][0]
                bg = self.P.grad[off:off + n_out]
            args.append((dY, X, self.P.g(wname), rows, n_out, n_in, ldy, ldx, bg))
        K.linear_dw_pair(*args)

    def join_side(self):
        """The caller's stream waits for every weight-gradient GEMM issued so far."""
        if self.side is not None:
            torch.cuda.current_stream().wait_stream(self.side)
            self.ws.busy.clear()

    def _db(self, dY, bname, rows, cols, ld=None):
        off = self.P.offsets[bname][0]
        K.colsum(dY, rows, cols, ld or cols, self.P.grad[off:off + cols])

    # ------------------------------------------------------------------ one transformer layer
    def layer_fwd(self, pre, x, B, Sx, L, pad, *, learned=0, cross=False, causal=False, ctx=None, heads, hd,
                  drop_p=0.0, seed=0, tag, out=None, window=0, fuse=False, h_in=None, next_ln=None, out_bf=None,
                  zsplice=None, ctx_ln=None):
        """TransformerLayer.forward (transformer_layer.py:44-61) on x f32 [B*Sx, d]. Returns the f32 output
        [B*Lq, d] and the saved state for layer_bwd. window > 0: sliding-window self-attention.

        fuse (no cross-attention): the two residual adds run in the fused residual + dropout + LayerNorm pass
        (svae_resid_ln_fwd) instead of the projection GEMMs' f32 epilogues -- the out-projection writes bf16 and the
        pass makes x1 = x + y and LayerNorm_f(x1); the FFN output is added (with its dropout) by the same pass fused
        with the NEXT layer's attention LayerNorm: next_ln = (LayerNorm name, z rows [B, d] f32, L, next tag) -- the z
        splice's rows are taken from the z rows -- which leaves (h, (x, mean, rstd)) in st['next_h'] for the next
        layer's h_in; without next_ln (the last layer) only the bf16 copy of the output is written, into out_bf (the
        head's input). ctx_ln = (cx, (ctx, mean, rstd)): this layer's context LayerNorm output, computed by the batched
        pass (ctx_ln_batched); its backward is then left to the caller (st['ctx_deferred'])."""
        d, ws, P = self.d, self.ws, self.P
        rows_x = B * Sx
        rot = self.rot(max(Sx, L), window)
        st = {'pre': pre, 'B': B, 'Sx': Sx, 'L': L, 'learned': learned, 'cross': cross, 'causal': causal,
              'heads': heads, 'hd': hd, 'drop_p': drop_p, 'seed': seed, 'x': x, 'tag': tag, 'window': window}
        a = pre + 'attention.'
        fuse = fuse and not cross
        if h_in is not None:
            h, st['ln_a'] = h_in
        else:   # (zsplice: the position-0 rows of x come from the batched z projections, svae_layernorm_fwd_z)
            h, st['ln_a'] = self._ln_fwd(pre + 'attn_layer_norm', x, rows_x, tag + '.ln_a', zsplice=zsplice)
        st['h'] = h
        pad_k = pad if Sx == L else None          # PaddedTensor getter: mask iff key length == L
        if learned:
            Lq = learned
            kv = ws.get(tag + '.kv', (rows_x, 2 * d))
            K.gemm(h, P.w(a + 'k_linear.weight'), kv, rows_x, 2 * d, d, epi=EPI_ROTARY_BF16,
                   bias=P.f(a + 'k_linear.bias'), rot=rot, rot_cols=d, rot_d=d, rot_seq=Sx)
            q = P.w(a + 'learned_queries').view(Lq, d)
            qargs = dict(sq=d, bq=0)
            kt, vt, sk = kv, kv[:, d:], 2 * d
            st['kv'] = kv
        else:
            Lq = Sx
            qkv = ws.get(tag + '.qkv', (rows_x, 3 * d))
            K.gemm(h, P.w(a + 'q_linear.weight'), qkv, rows_x, 3 * d, d, epi=EPI_ROTARY_BF16,
                   bias=P.f(a + 'q_linear.bias'), rot=rot, rot_cols=2 * d, rot_d=d, rot_seq=Sx)
            q = qkv
            qargs = dict(sq=3 * d, bq=Sx * 3 * d)
            kt, vt, sk = qkv[:, d:], qkv[:, 2 * d:], 3 * d
            st['qkv'] = qkv
        rows_q = B * Lq
        O = ws.get(tag + '.O', (rows_q, d))
        Ox = self._o_extra(tag + '.O', rows_q, d, Lq)
        lse = ws.get(tag + '.lse', (B, heads, Lq), f32)
        K.attention(q, kt, vt, O, lse, B=B, H=heads, Lq=Lq, Lk=Sx, hd=hd, so=d, bo=Lq * d, sk=sk, sv=sk,
                    bk=Sx * sk, bv=Sx * sk, key_pad=pad_k, causal=causal, window=window, **Ox, **qargs)
        st.update(O=O, Ox=Ox, lse=lse, Lq=Lq, pad_k=pad_k)
        resid = Lq == Sx                           # transformer_layer.py:49
        x1 = ws.get(tag + '.x1', (rows_q, d), f32)
        if fuse:
            # (the projection output stays f32: rounded to bf16 before the residual add it moved the C5-shape bottleneck
            # key gradient -- a cancellation residual -- past its 2 % parity bar)
            ya = ws.get('fuse.y', (rows_q, d), f32)
            K.gemm(O, P.w(a + 'output_linear.weight'), ya, rows_q, d, d, epi=EPI_F32, bias=P.f(a + 'output_linear.bias'))
            nm = pre + 'ffn_layer_norm'
            h2 = ws.get(tag + '.ln_f.y', (rows_q, d))
            mf, rf = ws.get(tag + '.ln_f.mean', (rows_q,), f32), ws.get(tag + '.ln_f.rstd', (rows_q,), f32)
            K.resid_ln_fwd(x if resid else None, ya, h2, rows_q, d, w=P.f(nm + '.weight'), b=P.f(nm + '.bias'), mean=mf,
                           rstd=rf, xo=x1)
            st['ln_f'] = (x1, mf, rf)
        else:
            K.gemm(O, P.w(a + 'output_linear.weight'), x1, rows_q, d, d, epi=EPI_F32,
                   bias=P.f(a + 'output_linear.bias'), resid=x if resid else None, ldr=d)
        st['resid'] = resid
        st['x1'] = x1
        xc = x1
        if cross:                                  # transformer_layer.py:51-54
            c = pre + 'cross_attention.'
            rows_c = B * L
            if ctx_ln is not None:
                cx, st['ln_ctx'] = ctx_ln
                st['ctx_deferred'] = True
            else:
                cx, st['ln_ctx'] = self._ln_fwd(pre + 'context_layer_norm', ctx, rows_c, tag + '.ln_ctx')
            hq, st['ln_cross'] = self._ln_fwd(pre + 'cross_attn_layer_norm', x1, rows_q, tag + '.ln_cross')
            qc = ws.get(tag + '.qc', (rows_q, d))
            K.gemm(hq, P.w(c + 'q_linear.weight'), qc, rows_q, d, d, epi=EPI_ROTARY_BF16, bias=P.f(c + 'q_linear.bias'),
                   rot=rot, rot_cols=d, rot_d=d, rot_seq=Lq)
            kvc = ws.get(tag + '.kvc', (rows_c, 2 * d))
            K.gemm(cx, P.w(c + 'k_linear.weight'), kvc, rows_c, 2 * d, d, epi=EPI_ROTARY_BF16,
                   bias=P.f(c + 'k_linear.bias'), rot=rot, rot_cols=d, rot_d=d, rot_seq=L)
            Oc = ws.get(tag + '.Oc', (rows_q, d))
            Ocx = self._o_extra(tag + '.Oc', rows_q, d, Lq)
            lsec = ws.get(tag + '.lsec', (B, heads, Lq), f32)
            K.attention(qc, kvc, kvc[:, d:], Oc, lsec, B=B, H=heads, Lq=Lq, Lk=L, hd=hd, sq=d, bq=Lq * d, sk=2 * d,
                        sv=2 * d, bk=L * 2 * d, bv=L * 2 * d, so=d, bo=Lq * d, key_pad=pad, causal=False, **Ocx)
            st['Ocx'] = Ocx
            x2 = ws.get(tag + '.x2', (rows_q, d), f32)
            K.gemm(Oc, P.w(c + 'output_linear.weight'), x2, rows_q, d, d, epi=EPI_F32,
                   bias=P.f(c + 'output_linear.bias'), resid=x1, ldr=d)
            st.update(cx=cx, hq=hq, qc=qc, kvc=kvc, Oc=Oc, lsec=lsec, x2=x2, pad_ctx=pad)
            xc = x2
        if not fuse:
            h2, st['ln_f'] = self._ln_fwd(pre + 'ffn_layer_norm', xc, rows_q, tag + '.ln_f')
        gprime = ws.get(tag + '.gprime', (rows_q, 4 * d))   # gelu'(pre-activation), saved by the epilogue
        f = ws.get(tag + '.f', (rows_q, 4 * d))
        K.gemm(h2, P.w(pre + 'ffn.0.weight'), f, rows_q, 4 * d, d, epi=EPI_GELU, bias=P.f(pre + 'ffn.0.bias'),
               aux=gprime, ldaux=4 * d)
        if fuse:
            yf = ws.get('fuse.y', (rows_q, d), f32)
            K.gemm(f, P.w(pre + 'ffn.2.weight'), yf, rows_q, d, 4 * d, epi=EPI_F32)
            if next_ln is not None:
                nm, zrows, zmod, ntag = next_ln
                out = ws.get(tag + '.out', (rows_q, d), f32) if out is None else out
                hn = ws.get(ntag + '.ln_a.y', (rows_q, d))
                mn, rn = ws.get(ntag + '.ln_a.mean', (rows_q,), f32), ws.get(ntag + '.ln_a.rstd', (rows_q,), f32)
                K.resid_ln_fwd(xc, yf, hn, rows_q, d, w=P.f(nm + '.weight'), b=P.f(nm + '.bias'), mean=mn, rstd=rn,
                               xo=out, drop_p=drop_p, seed=seed, zrows=zrows, zmod=zmod)
                st['next_h'] = (hn, (out, mn, rn))
            else:
                assert out_bf is not None, 'the last fused layer writes the bf16 copy of its output'
                K.resid_ln_fwd(xc, yf, out_bf, rows_q, d, xo=out, drop_p=drop_p, seed=seed)
        else:
            out = ws.get(tag + '.out', (rows_q, d), f32) if out is None else out
            # (out_bf: the last decoder layer's epilogue also writes the bf16 copy the vocabulary head reads)
            K.gemm(f, P.w(pre + 'ffn.2.weight'), out, rows_q, d, 4 * d, epi=EPI_DROPOUT_RESID, resid=xc, ldr=d,
                   drop_p=drop_p, seed=seed, aux=out_bf, ldaux=d if out_bf is not None else 0)
        st.update(h2=h2, gprime=gprime, f=f, xc=xc, rows_q=rows_q)
        return out, st

    def _o_extra(self, tag, rows_q, d, Lq):
        """The forward's extra copy of O for the backward's delta = rowsum(dO . O): the bf16 residual O - bf16(O)
        (o_lo, 2 B per element) by default; the f32 copy (o32) where the dO GEMM's delta epilogue reads it
        (SVAE_DELTA_FUSED=1) or SVAE_ATTN_O32=1. Keyword arguments for kernels.attention."""
        if self.delta_fused or self.o32_mode:
            return dict(o32=self.ws.get(tag + '32', (rows_q, d), f32), so32=d, bo32=Lq * d)
        return dict(o_lo=self.ws.get(tag + 'lo', (rows_q, d)), so_lo=d, bo_lo=Lq * d)

    def _dq_part(self, B, H, Lq, Lk, hd, window=0):
        """f32 workspace for the attention backward's per-key-block dQ partials (shared by all layers; window mode: the
        compact band planes, O(L) instead of O(L^2)))."""
        n = K.attn_dq_part_elems(B, H, Lq, Lk, hd, window)
        t = self.ws.bufs.get('b.dqpart')
        return t if t is not None and t.numel() >= n else self.ws.get('b.dqpart', (n,), f32)

    def layer_bwd(self, st, dout, dx_out, *, dx_accumulate=False, dctx=None, g2_ready=False, next_drop=None,
                  zsplice=None):
        """Backward of layer_fwd. dout f32 [B*Lq, d] (consumed as scratch). Writes d x into dx_out
        (accumulating into it when dx_accumulate and the layer has no residual); cross-attention context
        gradients accumulate into dctx. g2_ready: the dropout-masked bf16 dout is already in the 'b.g2' buffer
        (written by the previous layer_bwd's last LayerNorm backward); next_drop = (p, seed, zero_mod): this
        layer's last LayerNorm backward writes that buffer for the next layer_bwd (residual layers only).
        zsplice = (L, zrow, zrow_bf): that LayerNorm backward also moves rows r % L == 0 of dx_out into zrow / zrow_bf
        and zeroes them (the z splice's gradient, extract_rows + cast_bf16)."""
        d, ws, P = self.d, self.ws, self.P
        pre, B, Sx, L, Lq = st['pre'], st['B'], st['Sx'], st['L'], st['Lq']
        heads, hd = st['heads'], st['hd']
        rows_x, rows_q = B * Sx, st['rows_q']
        rot = self.rot(max(Sx, L), st['window'])
        a = pre + 'attention.'
        # ---- FFN (transformer_layer.py:56-61)
        g2 = ws.get('b.g2', (rows_q, d))
        if not g2_ready:
            K.dropout_bwd_cast(dout, g2, st['drop_p'], st['seed'], rows_q, d)
        dpre = ws.get('b.dpre', (rows_q, 4 * d))
        K.gemm(g2, P.wT(pre + 'ffn.2.weight', d, 4 * d), dpre, rows_q, 4 * d, d, epi=EPI_GELU_BWD, aux=st['gprime'],
               ldaux=4 * d)
        # (g2 stays intact until the next layer's backward)
        self._dw_pair((g2, st['f'], pre + 'ffn.2.weight', rows_q, d, 4 * d),
                      (dpre, st['h2'], pre + 'ffn.0.weight', rows_q, 4 * d, d, None, None, pre + 'ffn.0.bias'))
        dh2 = ws.get('b.dh2', (rows_q, d))
        K.gemm(dpre, P.wT(pre + 'ffn.0.weight', 4 * d, d), dh2, rows_q, d, 4 * d, epi=EPI_BF16)
        dxc = ws.get('b.dxc', (rows_q, d), f32)
        gxc = ws.get('b.gxc', (rows_q, d))
        self._ln_bwd(pre + 'ffn_layer_norm', dh2, st['ln_f'], rows_q, dout, dxc, gxc)
        dx1, gx1 = dxc, gxc
        if st['cross']:
            c = pre + 'cross_attention.'
            rows_c = B * L
            dOc = ws.get('b.dO', (rows_q, d))
            delta = ws.get('b.delta', (B, heads, Lq), f32)
            # the dO GEMM also writes delta = rowsum(dO . O) per head (its epilogue holds dO; no separate pass)
            K.gemm(gxc, P.wT(c + 'output_linear.weight', d, d), dOc, rows_q, d, d, epi=EPI_BF16, delta=delta if self.delta_fused else None,
                   delta_o32=st['Ocx'].get('o32'), ld_o32=d, delta_hd=hd, delta_seq=Lq)
            dqc = ws.get('b.dqc', (rows_q, d))
            dkvc = ws.get('b.dkvc', (rows_c, 2 * d))
            K.attention(st['qc'], st['kvc'], st['kvc'][:, d:], st['Oc'], st['lsec'], B=B, H=heads, Lq=Lq, Lk=L,
                        hd=hd, sq=d, bq=Lq * d, sk=2 * d, sv=2 * d, bk=L * 2 * d, bv=L * 2 * d, so=d, bo=Lq * d,
                        key_pad=st['pad_ctx'], causal=False, backward=True, delta_ready=self.delta_fused,
                        dout=dOc, sdo=d, bdo=Lq * d, delta=delta, dq_bf=dqc, ldq_bf=d, dk=dkvc, dv=dkvc[:, d:],
                        sdk=2 * d, sdv=2 * d, bdk=L * 2 * d, bdv=L * 2 * d, rot=rot, rot_d=d, **st['Ocx'],
                        dq_part=self._dq_part(B, heads, Lq, L, hd))
            self._dw_pair((gxc, st['Oc'], c + 'output_linear.weight', rows_q, d, d, None, None,
                           c + 'output_linear.bias'),
                          (dqc, st['hq'], c + 'q_linear.weight', rows_q, d, d, None, None, c + 'q_linear.bias'))
            dhq = ws.get('b.dhq', (rows_q, d))
            K.gemm(dqc, P.wT(c + 'q_linear.weight', d, d), dhq, rows_q, d, d, epi=EPI_BF16)
            self._dw(dkvc, st['cx'], c + 'k_linear.weight', rows_c, 2 * d, d, bias=c + 'k_linear.bias')
            # (a deferred context LayerNorm: its own gradient buffer, read by the batched backward after the layers)
            dcx = ws.get('b.dcx.' + st['tag'] if st.get('ctx_deferred') else 'b.dcx', (rows_c, d))
            K.gemm(dkvc, P.wT(c + 'k_linear.weight', 2 * d, d), dcx, rows_c, d, 2 * d, epi=EPI_BF16)
            dx1 = ws.get('b.dx1', (rows_q, d), f32)
            gx1 = ws.get('b.gx1', (rows_q, d))
            self._ln_bwd(pre + 'cross_attn_layer_norm', dhq, st['ln_cross'], rows_q, dxc, dx1, gx1)
            if st.get('ctx_deferred'):
                st['dcx'] = dcx
            else:
                self._ln_bwd(pre + 'context_layer_norm', dcx, st['ln_ctx'], rows_c, dctx, dctx)
        # ---- self / learned-query attention (attention.py:51-105)
        wo_dw = (gx1, st['O'], a + 'output_linear.weight', rows_q, d, d, None, None, a + 'output_linear.bias')
        dO = ws.get('b.dO', (rows_q, d))
        delta = ws.get('b.delta', (B, heads, Lq), f32)
        K.gemm(gx1, P.wT(a + 'output_linear.weight', d, d), dO, rows_q, d, d, epi=EPI_BF16, delta=delta if self.delta_fused else None,
               delta_o32=st['Ox'].get('o32'), ld_o32=d, delta_hd=hd, delta_seq=Lq)
        if st['learned']:
            kv = st['kv']
            dq32 = ws.get('b.dq32', (B * Lq, d), f32)
            dkv = ws.get('b.dkv', (rows_x, 2 * d))
            K.attention(P.w(a + 'learned_queries').view(Lq, d), kv, kv[:, d:], st['O'], st['lse'], B=B, H=heads,
                        Lq=Lq, Lk=Sx, hd=hd, sq=d, bq=0, sk=2 * d, sv=2 * d, bk=Sx * 2 * d, bv=Sx * 2 * d, so=d,
                        bo=Lq * d, key_pad=st['pad_k'], causal=False, backward=True, dout=dO, sdo=d, bdo=Lq * d,
                        delta=delta, delta_ready=self.delta_fused, dq=dq32, bdq=Lq * d, dk=dkv, dv=dkv[:, d:], sdk=2 * d, sdv=2 * d,
                        bdk=Sx * 2 * d, bdv=Sx * 2 * d, rot=rot, rot_d=d, **st['Ox'],
                        dq_part=self._dq_part(B, heads, Lq, Sx, hd))
            K.colsum(dq32, B, Lq * d, Lq * d, P.g(a + 'learned_queries').view(-1))
            self._dw_pair(wo_dw, (dkv, st['h'], a + 'k_linear.weight', rows_x, 2 * d, d, None, None,
                                  a + 'k_linear.bias'))
            dh = ws.get('b.dh', (rows_x, d))
            K.gemm(dkv, P.wT(a + 'k_linear.weight', 2 * d, d), dh, rows_x, d, 2 * d, epi=EPI_BF16)
        else:
            qkv = st['qkv']
            dqkv = ws.get('b.dqkv', (rows_x, 3 * d))
            K.attention(qkv, qkv[:, d:], qkv[:, 2 * d:], st['O'], st['lse'], B=B, H=heads, Lq=Lq, Lk=Sx, hd=hd,
                        sq=3 * d, bq=Sx * 3 * d, sk=3 * d, sv=3 * d, bk=Sx * 3 * d, bv=Sx * 3 * d, so=d, bo=Lq * d,
                        key_pad=st['pad_k'], causal=st['causal'], window=st['window'], backward=True, dout=dO,
                        sdo=d, bdo=Lq * d,
                        delta=delta, delta_ready=self.delta_fused, dq_bf=dqkv, ldq_bf=3 * d, dk=dqkv[:, d:], dv=dqkv[:, 2 * d:], sdk=3 * d,
                        sdv=3 * d, bdk=Sx * 3 * d, bdv=Sx * 3 * d, rot=rot, rot_d=d, **st['Ox'],
                        dq_part=self._dq_part(B, heads, Lq, Sx, hd, st['window']))
            self._dw_pair(wo_dw, (dqkv, st['h'], a + 'q_linear.weight', rows_x, 3 * d, d, None, None,
                                  a + 'q_linear.bias'))
            dh = ws.get('b.dh', (rows_x, d))
            K.gemm(dqkv, P.wT(a + 'q_linear.weight', 3 * d, d), dh, rows_x, d, 3 * d, epi=EPI_BF16)
        if st['resid']:
            # the next layer's dropout-masked bf16 dout and the z splice's rows ride along (no separate passes)
            self._ln_bwd(pre + 'attn_layer_norm', dh, st['ln_a'], rows_x, dx1, dx_out,
                         dx_bf=ws.get('b.g2', (rows_x, d)) if next_drop is not None else None, bf_drop=next_drop,
                         zsplice=zsplice)
            if dx_accumulate:
                raise NotImplementedError('residual + accumulate is handled by the caller')
        else:
            self._ln_bwd(pre + 'attn_layer_norm', dh, st['ln_a'], rows_x, dx_out if dx_accumulate else None, dx_out)

    # ------------------------------------------------------------------ full step
    def forward(self, ids, ntok, *, pad=True, eps=None, seed=0, kl_weight=1.0, dropout=0.1, need_logits=False):
        """TransformerVAE.training_step forward (transformer_vae.py:42-55). ids int [B, L] on the device."""
        hp, d, ws, P = self.hp, self.d, self.ws, self.P
        if not ids.is_cuda:
            raise RuntimeError('VAEEngine needs device tensors (no CPU fallback)')
        P.sync_shadow()
        B, L = ids.shape
        T, V, Z, N = B * L, hp.vocab_size, hp.latent_depth, hp.num_latents
        ids32 = ws.get('ids', (B, L), torch.int32)
        padm = None
        if pad is not None and pad is not False:
            padm = ws.get('pad', (B, L), torch.uint8)
        labels = ws.get('labels', (B, L), torch.int32)
        ntok64 = ws.get('ntok', (B,), torch.int64)
        if (self.small_fused and ids.dtype == torch.int64 and ids.is_contiguous() and isinstance(ntok, torch.Tensor) and ntok.is_cuda
                and ntok.dtype == torch.int64 and ntok.is_contiguous() and ntok.numel() == B
                and (padm is None or pad is True or (pad.dtype == torch.bool and pad.is_contiguous()))):
            # ids32, the next-token labels, the padding mask and the token counts in one launch
            K.prep_tokens(ids, pad if padm is not None else None, B, L, ids32, labels, padm, ntok, ntok64)
        else:
            ids32.copy_(ids)
            if padm is not None:
                padm.copy_(ids.eq(0) if pad is True else pad)
            labels[:, :-1].copy_(ids32[:, 1:])
            labels[:, -1] = 0
            ntok64.copy_(ntok)
        sv = {'B': B, 'L': L, 'dropout': dropout, 'seed': seed}

        x_emb = ws.get('x_emb', (T, d), f32)
        # (the decoder's input copy is written by the same gather: _decode's x_dec0)
        K.embedding_fwd(ids32, P.f('input_layer.0.weight'), x_emb, T, d, out2=ws.get('x_dec0', (T, d), f32))

        # ---- encoder (perceiver.py:39-50) + q(z|x) (conditional_gaussian.py:18)
        enc_bf, stats, sv['enc_layers'] = self._encode(x_emb, B, L, padm, dropout, seed)

        # ---- reparameterise + KL (conditional_gaussian.py:18-28, continuous_autoencoder.py:42-52)
        zf = ws.get('z', (B, Z), f32)
        zb = ws.get('z_bf', (B, Z))
        eps_buf = ws.get('eps', (B, Z), f32)
        raw_kl = ws.get('raw_kl', (B,), f32)
        kl = ws.get('kl', (2,), f32)
        if eps is not None:
            eps_buf.copy_(eps.reshape(B, Z))
        K.reparam_fwd(stats, eps_buf if eps is not None else None, _mix_seed(seed, 7), ntok64, zf, zb, eps_buf,
                      raw_kl, kl, B, Z)
        sv.update(enc_bf=enc_bf, stats=stats, z_bf=zb, eps=eps_buf)

        # ---- decoder (transformer_vae.py:85-93), position 0 replaced by z_projections[i](z) every layer
        xf, sv['dec_layers'] = self._decode(x_emb, zb, padm, B, L, dropout, seed, x_ready=True)

        # ---- output head + cross entropy (transformer_language_model.py:55-63, language_model.py:161-170)
        gp0 = ws.get('h0_gprime', (T, d))
        h0 = ws.get('h0', (T, d))
        K.gemm(xf, P.w('output_layer.0.weight'), h0, T, d, d, epi=EPI_GELU, bias=P.f('output_layer.0.bias'),
               aux=gp0, ldaux=d)
        hh, ln_h = self._ln_fwd('output_layer.2', h0, T, 'head.ln')
        nchunks, chunk_len = K.ce_chunking(B, L, V, CE_CHUNK_NUMEL)
        lse = ws.get('ce.lse', (T,), f32)
        row_loss = ws.get('ce.row_loss', (T,), f32)
        chunk_w = ws.get('ce.chunk_w', (max(8, nchunks),), f32)
        nll = ws.get('nll', (1,), f32)
        ntile = -(-V // 128)
        head = 'logits' if need_logits else self.head_mode
        W, bias = P.w('input_layer.0.weight'), P.f('output_layer.3.bias')
        logits = ws.get('logits', (T, V))          # the bf16 logits, or P = exp(logit - label logit)
        probe = self.probe
        if probe is not None:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
        if head == 'prob':
            coff = ws.get('ce.off', (T,), f32)
            K.ce_label_logit(hh, W, bias, labels, T, d, coff)
            part = ws.get('ce.psum', (ntile, T), f32)          # tile-major per-tile sums of P
            K.gemm(hh, W, logits, T, V, d, epi=EPI_CE_PROB, bias=bias, aux=part, labels=labels, row_a=coff)
        else:
            coff = None
            part = ws.get('ce.part', (T, ntile, 2), f32)
            lab_logit = ws.get('ce.label_logit', (T,), f32)
            K.gemm(hh, W, logits, T, V, d, epi=EPI_CE_STATS, bias=bias, aux=part, labels=labels, label_logit=lab_logit)
        if probe is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            probe.append((e0, e1))
        if head == 'prob':
            # rows whose P saturated (a logit > 88 nats above the label's) are recomputed exactly; their count
            # stays in ce_sat[0] (out['ce_saturated'])
            sat = ws.get('ce.sat', (T + 1,), torch.int32)
            K.ce_prob_finalize(part, ntile, coff, labels, T, L, nchunks, chunk_len, lse, row_loss, chunk_w, nll,
                               fix=(hh, W, bias, logits, sat))
        else:
            K.ce_finalize(part, ntile, lab_logit, labels, T, L, nchunks, chunk_len, lse, row_loss, chunk_w, nll)
        sv.update(xf=xf, gp0=gp0, h0=h0, hh=hh, ln_h=ln_h, logits=logits, lse=lse, chunk_w=chunk_w,
                  nchunks=nchunks, chunk_len=chunk_len, labels=labels, ids32=ids32, ntok=ntok64, x_emb=x_emb,
                  row_loss=row_loss, head=head, coff=coff)
        if self.small_fused:
            lbuf = ws.get('loss', (1,), f32)
            K.step_scalars(kl_weight, nll=nll, kl=kl, loss=lbuf)                  # transformer_vae.py:55
            loss = lbuf[0]
        else:
            loss = nll[0] + kl_weight * kl[0]
        self.saved = sv
        return {'loss': loss, 'nll': nll[0], 'kl': kl[0], 'train_kl': kl[1], 'raw_kl': raw_kl,
                'mu': stats[:, :Z], 'logvar': stats[:, Z:], 'stats': stats, 'kl_buf': kl, 'z': zf, 'eps': eps_buf,
                'logits': logits if need_logits else None,
                'ce_saturated': sat[0] if head == 'prob' else None}

    def weighted_nll(self, tok_w):
        """robust_cross_entropy(logits, labels, weight=tok_w) of the last forward (language_model.py:106-110, the
        val_bpb numerator) from its per-row losses: per chunk sum w[y] l / sum w[y], mean over chunks."""
        sv = self.saved
        out = torch.empty(1, dtype=f32, device=self.P.device)
        B, L = sv['B'], sv['L']
        K.ce_weighted_nll(sv['row_loss'], sv['labels'], tok_w, B * L, L, sv['nchunks'], sv['chunk_len'], out)
        return out[0]

    def _encode(self, x_emb, B, L, padm, dropout, seed):
        """Perceiver.forward (perceiver.py:39-50) then the q(z|x) linear (conditional_gaussian.py:18): returns
        the bf16 bottleneck [B, d], stats f32 [B, 2Z] = mu | logvar, and the layers' saved state."""
        hp, d, ws, P = self.hp, self.d, self.ws, self.P
        N, Z = hp.num_latents, hp.latent_depth
        lay = []
        z, st = self.layer_fwd('encoder.first_layer.', x_emb, B, L, L, padm, learned=N, heads=self.He, hd=64,
                               drop_p=dropout, seed=_mix_seed(seed, 1000), tag='e0')
        lay.append(st)
        nmid = hp.enc_layers - 2
        cxs = self._ctx_ln_fwd(x_emb, B * L, nmid) if P.ctx_batched else [None] * nmid
        for j in range(nmid):
            z, st = self.layer_fwd(f'encoder.middle_layers.{j}.', z, B, N, L, padm, cross=True, ctx=x_emb,
                                   heads=self.He, hd=64, drop_p=dropout, seed=_mix_seed(seed, 1001 + j), tag=f'e{j + 1}',
                                   ctx_ln=cxs[j])
            lay.append(st)
        enc, st = self.layer_fwd('encoder.bottleneck.', z, B, N, L, padm, learned=1, heads=self.He, hd=64,
                                 drop_p=dropout, seed=_mix_seed(seed, 1999), tag='eb')
        lay.append(st)
        enc_bf = ws.get('enc_bf', (B, d))
        K.cast_bf16(enc, enc_bf)
        stats = ws.get('stats', (B, 2 * Z), f32)
        K.gemm(enc_bf, P.w('q_of_z_given_x.linear.weight'), stats, B, 2 * Z, d, epi=EPI_F32,
               bias=P.f('q_of_z_given_x.linear.bias'))
        return enc_bf, stats, lay

    def _ctx_ln_fwd(self, x, rows, nmid):
        """Every middle layer's context_layer_norm(x_emb) (transformer_layer.py:52) in batched passes of <= LN_MULTI_MAX
        layers: returns per layer (cx bf16, (x, mean, rstd)) for layer_fwd's ctx_ln."""
        D, ws, P = self.d, self.ws, self.P
        mean = ws.get('ctx.ln.mean', (rows,), f32)
        rstd = ws.get('ctx.ln.rstd', (rows,), f32)
        out = []
        for j0 in range(0, nmid, LN_MULTI_MAX):
            js = range(j0, min(nmid, j0 + LN_MULTI_MAX))
            names = [f'encoder.middle_layers.{j}.context_layer_norm' for j in js]
            ys = [ws.get(f'e{j + 1}.ln_ctx.y', (rows, D)) for j in js]
            K.layernorm_fwd_multi(x, [P.f(n + '.weight') for n in names], [P.f(n + '.bias') for n in names], ys, mean,
                                  rstd, rows, D)
            out += [(y, (x, mean, rstd)) for y in ys]
        return out

    def _ctx_ln_bwd(self, sts, dctx):
        """The deferred context LayerNorm backwards of the middle layers' states sts (their dcx saved by layer_bwd), in
        batched passes of <= LN_MULTI_MAX: dctx += sum of their input gradients; each layer's affine gradients."""
        D, P = self.d, self.P
        for j0 in range(0, len(sts), LN_MULTI_MAX):
            grp = sts[j0:j0 + LN_MULTI_MAX]
            x, mean, rstd = grp[0]['ln_ctx']
            rows = x.shape[0]
            names = [g['pre'] + 'context_layer_norm' for g in grp]
            wgs = [P.grad[P.offsets[n + '.weight'][0]:][:2 * D] for n in names]
            n1 = 1024 * 2 * D
            if self.cs_batch:
                if len(self._cs_pending) + len(grp) > COLSUM_MAX:
                    self.flush_colsum()
                k = len(self._cs_pending)
                part = self.ws.get('ln.parts', (COLSUM_MAX * n1,), f32)[k * n1:(k + len(grp)) * n1]
                defer = self._cs_pending
            else:
                part = self.ws.get('ln.partm', (LN_MULTI_MAX * n1,), f32)
                defer = None
            K.layernorm_bwd_multi([g['dcx'] for g in grp], x, [P.f(n + '.weight') for n in names], mean, rstd, dctx,
                                  dctx, wgs, rows, D, part, defer=defer)

    def _inputs(self, ids, pad):
        """ids [B, L] -> (int32 ids, uint8 key-padding mask or None) in the workspace."""
        B, L = ids.shape
        ids32 = self.ws.get('ids', (B, L), torch.int32)
        ids32.copy_(ids)
        padm = None
        if pad is not None and pad is not False:
            padm = self.ws.get('pad', (B, L), torch.uint8)
            padm.copy_(ids.eq(0) if pad is True else pad)
        return ids32, padm

    def mutual_info(self, out, eps=None, num_samples=10):
        """kl - marginal_kl(q) for the step's posterior (transformer_vae.py:59-61, math_utils.py:51-58) in one
        fused kernel pair; eps [num_samples, B, Z] f32 or None (drawn in-kernel from a torch-RNG seed).
        Returns a fresh 0-d f32 tensor (the step's workspace is reused by the next step)."""
        stats = out['stats']
        B, Z = stats.shape[0], stats.shape[1] // 2
        if eps is not None:
            eps = eps.to(stats.device, f32).reshape(num_samples, B, Z).contiguous()
        ws = self.ws.get('mi_ws', (2 * num_samples * B,), f32)
        res = torch.empty((), dtype=f32, device=stats.device)
        seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        K.mutual_info(stats, out['kl_buf'], B, Z, seed, res, ws, eps=eps, S=num_samples)
        return res

    def posterior(self, ids, pad=True):
        """q(z|x) without the decoder (transformer_vae.py:73-74, :81-83): stats f32 [B, 2Z] = mu | logvar."""
        if not ids.is_cuda:
            raise RuntimeError('VAEEngine needs device tensors (no CPU fallback)')
        self.P.sync_shadow()
        B, L = ids.shape
        ids32, padm = self._inputs(ids, pad)
        x_emb = self.ws.get('x_emb', (B * L, self.d), f32)
        K.embedding_fwd(ids32, self.P.f('input_layer.0.weight'), x_emb, B * L, self.d)
        _, stats, _ = self._encode(x_emb, B, L, padm, 0.0, 0)
        return stats

    def seq_log_prob(self, x_emb, labels, z, pad=None, max_tokens=32768):
        """log p(x|z) summed over each sequence (continuous_autoencoder.py:82-88). x_emb f32 [G, B, L, d] (the
        embedded input; any strides — the IW estimate passes the batch expanded over G samples, copied one
        sub-batch at a time, never materialised), labels int [G, B, L-1] (label 0 adds 0), z f32 [G, B, Z],
        pad [G, B, L] bool key-padding mask or None. Returns f32 [G, B]. Sub-batches hold <= max_tokens tokens
        (whole groups when B * L fits); the vocabulary GEMM keeps only its CE statistics."""
        hp, d, ws, P = self.hp, self.d, self.ws, self.P
        if not x_emb.is_cuda:
            raise RuntimeError('VAEEngine needs device tensors (no CPU fallback)')
        P.sync_shadow()
        G, Bt, L = x_emb.shape[0], x_emb.shape[1], x_emb.shape[2]
        V, Z = hp.vocab_size, hp.latent_depth
        out = torch.empty(G, Bt, dtype=f32, device=P.device)
        ntile = -(-V // 128)
        if Bt * L <= max_tokens:
            gstep, bstep = max(1, max_tokens // (Bt * L)), Bt
        else:
            gstep, bstep = 1, max(1, max_tokens // L)
        for g0 in range(0, G, gstep):
            g1 = min(G, g0 + gstep)
            for b0 in range(0, Bt, bstep):
                b1 = min(Bt, b0 + bstep)
                ng, nb = g1 - g0, b1 - b0
                B = ng * nb
                T = B * L
                padm = None
                if pad is not None:
                    padm = ws.get('pad', (B, L), torch.uint8)
                    padm.view(ng, nb, L).copy_(pad[g0:g1, b0:b1])
                lab = ws.get('labels', (B, L), torch.int32)
                lab.view(ng, nb, L)[:, :, :-1].copy_(labels[g0:g1, b0:b1])
                lab[:, -1] = 0
                xe = ws.get('x_emb', (T, d), f32)
                xe.view(ng, nb, L, d).copy_(x_emb[g0:g1, b0:b1])
                zf = ws.get('z_f32', (B, Z), f32)
                zf.view(ng, nb, Z).copy_(z[g0:g1, b0:b1])
                zb = ws.get('z_bf', (B, Z))
                K.cast_bf16(zf, zb)
                xf, _ = self._decode(xe, zb, padm, B, L, 0.0, 0)
                hh = self._head_hidden(xf, T)
                part = ws.get('ce.part', (T, ntile, 2), f32)
                lab_logit = ws.get('ce.label_logit', (T,), f32)
                K.gemm(hh, P.w('input_layer.0.weight'), None, T, V, d, epi=EPI_CE_STATS,
                       bias=P.f('output_layer.3.bias'), aux=part, labels=lab, label_logit=lab_logit)
                res = ws.get('seq_lp', (B,), f32)
                K.ce_seq_logprob(part, ntile, lab_logit, lab, T, L, res)
                out[g0:g1, b0:b1].copy_(res.view(ng, nb))
        return out

    def _head_hidden(self, xf, T):
        """output_layer[:3] (transformer_language_model.py:55-61): LayerNorm(GELU(Linear(x))) as the bf16
        operand of the tied vocabulary GEMM, from the decoder's bf16 output xf."""
        d, ws, P = self.d, self.ws, self.P
        gp0 = ws.get('h0_gprime', (T, d))
        h0 = ws.get('h0', (T, d))
        K.gemm(xf, P.w('output_layer.0.weight'), h0, T, d, d, epi=EPI_GELU, bias=P.f('output_layer.0.bias'),
               aux=gp0, ldaux=d)
        hh, _ = self._ln_fwd('output_layer.2', h0, T, 'head.ln')
        return hh

    def _decode(self, x_emb, zb, padm, B, L, dropout, seed, x_ready=False):
        """The decoder stack of reconstruct (transformer_vae.py:85-93). Returns the bf16 copy of the last layer's
        output [T, d] (the head's input; its f32 is not needed by any pass) and the layers' saved state.
        Position 0 of every layer's input is z_projections[i](z): for layer 0 written into the embedding copy, for
        the later layers into a [B, d] buffer the fused residual + LayerNorm pass of the layer below takes those rows
        from (SVAE_FUSE_LN=0: the round-2 path, f32 GEMM epilogues + separate LayerNorms, for A/B runs)."""
        hp, d, ws, P = self.hp, self.d, self.ws, self.P
        T, Z = B * L, hp.latent_depth
        if self.window and L % 32:
            raise ValueError(f'sparse decoder attention needs seq_len % 32 == 0 (SparseAttention block_size 32, '
                             f'sparse_attention.py:81), got {L}')
        fuse = self.fuse_ln
        xs = ws.get('x_dec0', (T, d), f32)
        if not x_ready:   # (the training forward's embedding gather wrote it already)
            xs.copy_(x_emb)
        xf = ws.get('xf_bf', (T, d))
        dec = []
        h_in = None
        # (zf_batch: every layer's z projection in one launch, spliced in by the layer's first LayerNorm)
        # (the launch takes <= ZPROJ_MAX layers and a latent of <= 1024: deeper models run it in chunks, wider latents
        # the per-layer GEMM path)
        zf_batch = self.zf_batch and not fuse and d % 8 == 0 and Z <= 1024
        if zf_batch:
            zall = ws.get('zproj_all', (hp.num_layers, B, d), f32)
            segs = [(P.w(f'z_projections.{i}.weight'), P.f(f'z_projections.{i}.bias'), zall[i])
                    for i in range(hp.num_layers)]
            for c0 in range(0, len(segs), ZPROJ_MAX):
                K.zproj_fwd_multi(segs[c0:c0 + ZPROJ_MAX], zb, B, d, Z)
        else:
            K.gemm(zb, P.w('z_projections.0.weight'), xs, B, d, Z, ldc=L * d, epi=EPI_F32,
                   bias=P.f('z_projections.0.bias'))
        for i in range(hp.num_layers):
            last = i + 1 == hp.num_layers
            if fuse:
                nxt = None
                if not last:
                    zrows = ws.get('zrows', (B, d), f32)
                    K.gemm(zb, P.w(f'z_projections.{i + 1}.weight'), zrows, B, d, Z, epi=EPI_F32,
                           bias=P.f(f'z_projections.{i + 1}.bias'))
                    nxt = (f'decoder_layers.{i + 1}.attn_layer_norm', zrows, L, f'd{i + 1}')
                out = None if last else ws.get(f'x_dec{i + 1}', (T, d), f32)
            else:
                if i > 0 and not zf_batch:
                    K.gemm(zb, P.w(f'z_projections.{i}.weight'), xs, B, d, Z, ldc=L * d, epi=EPI_F32,
                           bias=P.f(f'z_projections.{i}.bias'))
                nxt, out = None, ws.get(f'x_dec{i + 1}', (T, d), f32)
            xs, st = self.layer_fwd(f'decoder_layers.{i}.', xs, B, L, L, padm, causal=True, heads=self.H,
                                    hd=self.hd, drop_p=dropout, seed=_mix_seed(seed, i), tag=f'd{i}', out=out,
                                    window=self.window, fuse=fuse, h_in=h_in, next_ln=nxt,
                                    out_bf=xf if last and (fuse or self.resid_bf16) else None,
                                    zsplice=(zall[i], L) if zf_batch else None)
            h_in = st.pop('next_h', None)
            dec.append(st)
        if not fuse and not self.resid_bf16:
            K.cast_bf16(xs, xf)
        return xf, dec

    def reconstruct_f32(self, x_emb, z, pad=None):
        """reconstruct() in the fp32 kernel mode (f32-input MFMA GEMMs, f32 attention / LayerNorm): logits
        [B, L, V] f32 for the bit-exact argmax check against the fp32 reference."""
        hp, d, P = self.hp, self.d, self.P
        dev = P.device
        B, L = x_emb.shape[0], x_emb.shape[1]
        T, V, Z, H, hd = B * L, hp.vocab_size, hp.latent_depth, self.H, self.hd
        rot = self.rot(L, self.window)
        padm = None
        if pad is not None:
            padm = torch.empty(B, L, dtype=torch.uint8, device=dev)
            padm.copy_(pad)
        x = x_emb.reshape(T, d).clone()
        h = torch.empty(T, d, device=dev)
        qkv = torch.empty(T, 3 * d, device=dev)
        o = torch.empty(T, d, device=dev)
        x1 = torch.empty(T, d, device=dev)
        f = torch.empty(T, 4 * d, device=dev)
        for i in range(hp.num_layers):
            pre = f'decoder_layers.{i}.'
            a = pre + 'attention.'
            # position 0 <- z_projections[i](z)   (transformer_vae.py:89-90)
            K.gemm_f32(z, P.f(f'z_projections.{i}.weight'), x, B, d, Z, ldc=L * d, bias=P.f(f'z_projections.{i}.bias'))
            K.layernorm_fwd_f32(x, P.f(pre + 'attn_layer_norm.weight'), P.f(pre + 'attn_layer_norm.bias'), h, T, d)
            K.gemm_f32(h, P.f(a + 'q_linear.weight'), qkv, T, 3 * d, d, epi=EPI_ROTARY_BF16, bias=P.f(a + 'q_linear.bias'),
                       rot=rot, rot_cols=2 * d, rot_d=d, rot_seq=L)
            K.attention_f32(qkv, qkv[:, d:], qkv[:, 2 * d:], o, B=B, H=H, Lq=L, Lk=L, hd=hd, sq=3 * d, sk=3 * d,
                            sv=3 * d, so=d, bq=L * 3 * d, bk=L * 3 * d, bv=L * 3 * d, bo=L * d, key_pad=padm, causal=True,
                            window=self.window)
            K.gemm_f32(o, P.f(a + 'output_linear.weight'), x1, T, d, d, bias=P.f(a + 'output_linear.bias'), resid=x, ldr=d)
            K.layernorm_fwd_f32(x1, P.f(pre + 'ffn_layer_norm.weight'), P.f(pre + 'ffn_layer_norm.bias'), h, T, d)
            K.gemm_f32(h, P.f(pre + 'ffn.0.weight'), f, T, 4 * d, d, epi=EPI_GELU, bias=P.f(pre + 'ffn.0.bias'))
            K.gemm_f32(f, P.f(pre + 'ffn.2.weight'), x, T, d, 4 * d, resid=x1, ldr=d)
        h0 = torch.empty(T, d, device=dev)
        K.gemm_f32(x, P.f('output_layer.0.weight'), h0, T, d, d, epi=EPI_GELU, bias=P.f('output_layer.0.bias'))
        K.layernorm_fwd_f32(h0, P.f('output_layer.2.weight'), P.f('output_layer.2.bias'), h, T, d)
        logits = torch.empty(B, L, V, device=dev)
        K.gemm_f32(h, P.f('input_layer.0.weight'), logits, T, V, d, bias=P.f('output_layer.3.bias'))
        return logits

    def reconstruct(self, x_emb, z, pad=None):
        """TransformerVAE.reconstruct (transformer_vae.py:85-93): decoder + head logits [B, L, V] bf16 from
        x_emb f32 [B, L, d] and z f32 [B, latent]; pad = [B, L] mask or None."""
        hp, d, ws, P = self.hp, self.d, self.ws, self.P
        P.sync_shadow()
        B, L = x_emb.shape[0], x_emb.shape[1]
        T, V, Z = B * L, hp.vocab_size, hp.latent_depth
        padm = None
        if pad is not None:
            padm = ws.get('pad', (B, L), torch.uint8)
            padm.copy_(pad)
        zb = ws.get('z_bf', (B, Z))
        K.cast_bf16(z, zb)
        xf, _ = self._decode(x_emb.reshape(T, d), zb, padm, B, L, 0.0, 0)
        gp0 = ws.get('h0_gprime', (T, d))
        h0 = ws.get('h0', (T, d))
        K.gemm(xf, P.w('output_layer.0.weight'), h0, T, d, d, epi=EPI_GELU, bias=P.f('output_layer.0.bias'),
               aux=gp0, ldaux=d)
        hh, _ = self._ln_fwd('output_layer.2', h0, T, 'head.ln')
        logits = torch.empty(B, L, V, dtype=bf16, device=P.device)
        K.gemm(hh, P.w('input_layer.0.weight'), logits, T, V, d, epi=EPI_BF16, bias=P.f('output_layer.3.bias'))
        return logits

    def backward(self, gloss, kl_weight, ready=None):
        """Gradients of loss = nll + kl_weight * kl into the flat gradient arena (accumulating). `ready(end)`
        is called each time the arena prefix [0, end) holds final gradients (data-parallel bucketing)."""
        sv, hp, d, ws, P = self.saved, self.hp, self.d, self.ws, self.P
        user_ready = ready

        def ready(end):                     # a bucket's gradients must be complete before its all-reduce
            if user_ready is not None:
                self.flush_colsum()
                self.flush_zproj()
                self.join_side()
                user_ready(end)
        if sv is None:
            raise RuntimeError('backward() without a saved forward')
        B, L = sv['B'], sv['L']
        T, V, Z, N = B * L, hp.vocab_size, hp.latent_depth, hp.num_latents
        gs = ws.get('gscale', (2,), f32)
        gl = gloss.reshape(1)
        if self.small_fused and gl.is_cuda and gl.dtype == f32:
            K.step_scalars(kl_weight, gloss=gl, gs=gs)
        else:
            gs[0:1].copy_(gl)
            gs[1:2].copy_(gl * kl_weight)

        # ---- head
        logits = sv['logits']
        dhh = ws.get('b.dhh', (T, d))
        nch, clen = sv['nchunks'], sv['chunk_len']
        if sv['head'] == 'prob':
            # dlogits = r (x) P - q (x) onehot, never formed: dW = P^T (r . hh) (+ one-hot part in the embedding
            # backward), d bias = sum_t r_t P[t] (weighted row sums of the dW GEMM) - q at the labels (prep),
            # dX = r . (P W) - q W[label]
            hh = sv['hh']
            hh_r = ws.get('b.hh_r', (T, d))
            r_t = ws.get('b.ce_r', (T,), f32)
            q_t = ws.get('b.ce_q', (T,), f32)
            dbias = P.g('output_layer.3.bias')
            K.ce_prob_bwd_prep(hh, sv['lse'], sv['coff'], sv['chunk_w'], sv['labels'], gs[0:1], T, L, nch, clen, d, hh_r,
                               r_t, q_t, dbias)
            # (a K-contiguous B, (r . hh)^T, measured the same: 1069 vs 1079 us; the k-weighted row sums cost ~15 %)
            s = self._head_dw_splits(V, d)
            if s == 1:
                K.gemm(logits, hh_r, P.g('input_layer.0.weight'), V, d, T, a_t=True, b_t=True, lda=V, ldb=d, ldc=d,
                       epi=EPI_F32_ACC, a_rowsum=dbias, k_weight=r_t)
            else:   # split-K slabs (deterministic C), summed into the gradient by slab_reduce
                slab = ws.get('b.head_dw_slab', (s * V * d,), f32)
                K.gemm(logits, hh_r, P.g('input_layer.0.weight'), V, d, T, a_t=True, b_t=True, lda=V, ldb=d, ldc=d,
                       epi=EPI_F32_ATOMIC, splits=s, aux=slab, a_rowsum=dbias, k_weight=r_t)
            W = P.w('input_layer.0.weight')
            K.gemm(logits, P.wT('input_layer.0.weight', V, d), dhh, T, d, V, epi=EPI_ROWSCALE_GATHER,
                   labels=sv['labels'], row_a=r_t, row_b=q_t, gather=W, ldg=d)
            sv['ce_q'] = q_t
        else:
            K.ce_grad(logits, V, sv['lse'], sv['chunk_w'], sv['labels'], gs[0:1], T, V, L, nch, clen)
            # (the vocabulary-head dW stays in order: next to the equally large head dX it only contends)
            self._dw(logits, sv['hh'], 'input_layer.0.weight', T, V, d, bias='output_layer.3.bias', on_side=False)
            K.gemm(logits, P.wT('input_layer.0.weight', V, d), dhh, T, d, V, epi=EPI_BF16)
        dpre0 = ws.get('b.dpre0', (T, d))
        if self.ln_gelu:   # the head LayerNorm's backward and the GELU backward before it in one pass
            self._ln_bwd('output_layer.2', dhh, sv['ln_h'], T, None, None, dx_bf=dpre0, gelu=sv['gp0'])
        else:
            dh0 = ws.get('b.dh0', (T, d), f32)
            self._ln_bwd('output_layer.2', dhh, sv['ln_h'], T, None, dh0)
            K.gelu_bwd(dh0, sv['gp0'], dpre0, T * d)
        self._dw(dpre0, sv['xf'], 'output_layer.0.weight', T, d, d, bias='output_layer.0.bias')
        dx = ws.get('b.dx_dec', (T, d), f32)
        # (the same epilogue writes the top decoder layer's dropout-masked bf16 FFN-output gradient, b.g2: no
        # separate dropout_bwd_cast pass over [T, d]; SVAE_HEAD_G2=0 for A/B runs)
        top = sv['dec_layers'][-1]
        g2_pre = self.head_g2 and top['rows_q'] == T
        K.gemm(dpre0, P.wT('output_layer.0.weight', d, d), dx, T, d, d, epi=EPI_F32,
               aux=ws.get('b.g2', (T, d)) if g2_pre else None, ldaux=d if g2_pre else 0,
               drop_p=top['drop_p'] if g2_pre else 0.0, seed=top['seed'] if g2_pre else 0)
        ready(P.end('output_layer.3.bias'))

        # ---- decoder layers, last to first
        dz = ws.get('b.dz', (B, Z), f32, zero=True)
        dzh = ws.get('b.dzh', (B, d), f32)
        dzh_bf = ws.get('b.dzh_bf', (B, d))
        dx_prev = ws.get('b.dx_prev', (T, d), f32)
        g2_ready = g2_pre
        for i in reversed(range(hp.num_layers)):
            st = sv['dec_layers'][i]
            # the next (lower) layer's FFN dropout backward + position-0 zeroing (extract_rows below) fused into this
            # layer's last LayerNorm backward (same rows: a residual layer maps B*L rows to B*L rows)
            nd = None
            if i > 0 and st['resid'] and sv['dec_layers'][i - 1]['rows_q'] == T:
                nst = sv['dec_layers'][i - 1]
                nd = (nst['drop_p'], nst['seed'], L)
            # position-0 splice: its gradient feeds z_projections[i]; earlier layers see zero there (moved out of dx by
            # the layer's last LayerNorm backward when it is a residual layer)
            dzh_i = ws.get('b.dzh_all', (hp.num_layers, B, d), f32)[i] if self.zp_batch else dzh
            zs = (L, dzh_i, None) if st['resid'] and st['rows_q'] == T else None
            self.layer_bwd(st, dx, dx_prev, g2_ready=g2_ready, next_drop=nd, zsplice=zs)
            g2_ready = nd is not None
            wz, bz = f'z_projections.{i}.weight', f'z_projections.{i}.bias'
            if zs is not None and self.zp_batch:
                # dW, d bias and dz of z_projections[i]: deferred, then every layer's in one launch (flush_zproj, also
                # at each data-parallel bucket point); dz sums the layers in this loop's order either way
                if len(self._zp_pending) == ZPROJ_MAX:
                    self.flush_zproj()
                self._zp_ctx = (sv['z_bf'], dz, B, d, Z)
                self._zp_pending.append((dzh_i, P.w(wz), P.g(wz), P.g(bz)))
            elif zs is not None:   # dW, d bias and dz of z_projections[i] in one f32 launch
                K.zproj_bwd(dzh, sv['z_bf'], P.w(wz), P.g(wz), P.g(bz), dz, B, d, Z)
            else:
                self.flush_zproj()
                K.extract_rows(dx_prev, d, T, L, d, dzh)
                K.cast_bf16(dzh, dzh_bf)
                self._dw(dzh_bf, sv['z_bf'], wz, B, d, Z, bias=bz)   # (bias gradient = the fused row sums)
                # dz += dzh . W_i: a 64 x 64 output over K = d -> split K over blocks (f32 atomics into dz)
                K.gemm(dzh_bf, P.w(wz), dz, B, Z, d, b_t=True, epi=EPI_F32_ATOMIC, splits=max(1, min(8, d // 64)))
            ready(P.end(f'z_projections.{i}.bias'))
            dx, dx_prev = dx_prev, dx
        self.flush_zproj()                            # (before reparam_bwd reads dz)
        dx_emb = dx                                   # decoder part of d x_emb (rows 0 already zero)

        # ---- reparameterise + q(z|x)
        dstats = ws.get('b.dstats', (B, 2 * Z), f32)
        K.reparam_bwd(sv['stats'], sv['eps'], dz, sv['ntok'], gs[1:2], dstats, B, Z)
        dstats_bf = ws.get('b.dstats_bf', (B, 2 * Z))
        K.cast_bf16(dstats, dstats_bf)
        self._dw(dstats_bf, sv['enc_bf'], 'q_of_z_given_x.linear.weight', B, 2 * Z, d)
        self._db(dstats, 'q_of_z_given_x.linear.bias', B, 2 * Z)
        denc = ws.get('b.denc', (B, d), f32)
        K.gemm(dstats_bf, P.w('q_of_z_given_x.linear.weight'), denc, B, d, 2 * Z, b_t=True, epi=EPI_F32)
        ready(P.end('q_of_z_given_x.linear.bias'))

        # ---- encoder, bottleneck -> middle -> first
        enc = sv['enc_layers']
        dcur = denc
        for k in reversed(range(1, len(enc))):
            st = enc[k]
            nxt = ws.get(f'b.denc{k}', (B * N, d), f32)
            self.layer_bwd(st, dcur, nxt, dctx=dx_emb)
            ready(P.end(st['pre'] + 'ffn_layer_norm.bias'))
            dcur = nxt
        deferred = [st for st in enc if st.get('ctx_deferred')]
        if deferred:   # the batched context LayerNorm backward (ctx_ln_batched); its parameters come next in the layout
            self._ctx_ln_bwd(deferred[::-1], dx_emb)
            ready(P.end(deferred[0]['pre'] + 'context_layer_norm.bias'))
        st0 = enc[0]
        if st0['resid']:   # L == num_latents: the first layer keeps its residual (transformer_layer.py:49)
            tmp = ws.get('b.dfirst', (T, d), f32)
            self.layer_bwd(st0, dcur, tmp)
            self.join_side()        # the tied weight's head gradient (side stream) before the scatter-add
            K.embedding_bwd(sv['ids32'], tmp, P.g('input_layer.0.weight'), T, d)   # (the head's part: below)
        else:
            self.layer_bwd(st0, dcur, dx_emb, dx_accumulate=True)

        ready(P.end('encoder.first_layer.ffn_layer_norm.bias'))
        # ---- embedding (tied with the head weight)
        self.join_side()            # the tied weight's head gradient (side stream) before the scatter-add
        self._embedding_bwd(sv, dx_emb, T, d)
        ready(P.n_live)
        self.flush_colsum()
        self.join_side()

    def _embedding_bwd(self, sv, dx, T, d):
        """Scatter-add of d x_emb into the tied table; with the P-head, fused with the head's one-hot dW part."""
        if sv['head'] == 'prob':
            K.embedding_bwd_ce(sv['ids32'], dx, self.P.g('input_layer.0.weight'), T, d, sv['L'], sv['hh'], sv['ce_q'])
        else:
            K.embedding_bwd(sv['ids32'], dx, self.P.g('input_layer.0.weight'), T, d)
