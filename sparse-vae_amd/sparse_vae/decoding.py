"""KV-cache decoding of TransformerVAE.sample (transformer_vae.py:95-128) on libsvae, in f32.

One decode step = for every decoder layer: LayerNorm -> fused q|k|v linear with rotary at position cur-1 ->
cache append + attention over the visible keys -> output linear (+ residual) -> LayerNorm -> FFN (GELU) (+
residual); then the output head (Linear, GELU, LayerNorm, tied vocabulary Linear), the repetition penalty
and the sampler, which writes the next id and the live mask, and `cur += 1`. Every kernel reads the position
from the device scalar `cur`, so the step for positions >= 2 is captured once as a HIP graph
(torch.cuda.CUDAGraph) and replayed. Step 1 differs (each layer's input is z_projections[i](z),
transformer_vae.py:119-121) and runs eagerly.

Finished rows are not compacted as the reference does (Attention.update_kv_cache, attention.py:162-168): their
ids stop changing (the sampler skips rows whose live flag is clear), which keeps the step's shapes fixed for
the graph. Rows are independent, so the surviving rows' outputs are the same.

The KV cache holds every position ([layers][B][H][T][hd] f32); with sparse_self_attention the attention kernel
reads exactly the keys the reference's sliding-window cache keeps (attention.py:115-140).
"""
import torch

from . import kernels as K
from ._native import EPI_F32, EPI_GELU, EPI_ROTARY_BF16

f32 = torch.float32


class KVDecoder:
    def __init__(self, engine, state, z, use_graph=True):
        self.eng, self.st = engine, state
        P, hp = engine.P, engine.hp
        self.P = P
        B, T = state.output_ids.shape
        d, H, NL, V = engine.d, engine.H, hp.num_layers, hp.vocab_size
        self.B, self.T, self.d, self.H, self.hd, self.NL, self.V = B, T, d, H, engine.hd, NL, V
        self.window = engine.window
        dev = P.device
        self.z = z.reshape(B, -1).to(dev, f32).contiguous()
        self.kc = torch.empty(NL, B, H, T, self.hd, device=dev, dtype=f32)
        self.vc = torch.empty_like(self.kc)
        self.rot = engine.rot(T, self.window)
        e = lambda *s: torch.empty(*s, device=dev, dtype=f32)   # noqa: E731
        self.x, self.xin, self.h, self.x1 = e(B, d), e(B, d), e(B, d), e(B, d)
        self.qkv, self.O, self.f = e(B, 3 * d), e(B, d), e(B, 4 * d)
        self.h0, self.hh, self.logits = e(B, d), e(B, d), e(B, V)
        self.part = e(16 * B * 4 * d)          # split-K partials of the narrow linears (<= 16 splits)
        self.use_graph = use_graph
        self.graph = None

    # ------------------------------------------------------------------ one layer (transformer_layer.py:44-61)
    def _layer(self, i, x_in, x_out):
        P, B, d, st = self.P, self.B, self.d, self.st
        pre = f'decoder_layers.{i}.'
        a = pre + 'attention.'
        K.layernorm_fwd_f32(x_in, P.f(pre + 'attn_layer_norm.weight'), P.f(pre + 'attn_layer_norm.bias'), self.h, B, d)
        # q | k | v weights and biases are adjacent in the arena: one [3d, d] operand; rotary on q and k
        K.dec_linear(self.h, P.f(a + 'q_linear.weight'), self.qkv, B, 3 * d, d, bias=P.f(a + 'q_linear.bias'),
                     epi=EPI_ROTARY_BF16, rot=self.rot, rot_cols=2 * d, rot_d=d, cur=st.cur, part=self.part)
        K.dec_attn(self.qkv, self.kc[i], self.vc[i], self.O, B, self.H, self.hd, self.T, st.cur, self.window)
        K.dec_linear(self.O, P.f(a + 'output_linear.weight'), self.x1, B, d, d, bias=P.f(a + 'output_linear.bias'),
                     resid=x_in, part=self.part)
        K.layernorm_fwd_f32(self.x1, P.f(pre + 'ffn_layer_norm.weight'), P.f(pre + 'ffn_layer_norm.bias'), self.h, B, d)
        K.dec_linear(self.h, P.f(pre + 'ffn.0.weight'), self.f, B, 4 * d, d, bias=P.f(pre + 'ffn.0.bias'), epi=EPI_GELU,
                     part=self.part)
        K.dec_linear(self.f, P.f(pre + 'ffn.2.weight'), x_out, B, d, 4 * d, resid=self.x1, part=self.part)

    def _step(self, first):
        P, B, d, st = self.P, self.B, self.d, self.st
        Z = self.z.shape[1]
        if not first:
            K.dec_embed(st.output_ids, self.T, st.cur, P.f('input_layer.0.weight'), self.x, B, d)
        for i in range(self.NL):
            if first:    # transformer_vae.py:119-120: the layer input is z_projections[i](z) at current_index 1
                K.dec_linear(self.z, P.f(f'z_projections.{i}.weight'), self.xin, B, d, Z,
                             bias=P.f(f'z_projections.{i}.bias'))
                self._layer(i, self.xin, self.x)
            else:
                self._layer(i, self.x, self.x)
        # output_layer (transformer_language_model.py:55-63)
        K.dec_linear(self.x, P.f('output_layer.0.weight'), self.h0, B, d, d, bias=P.f('output_layer.0.bias'),
                     epi=EPI_GELU, part=self.part)
        K.layernorm_fwd_f32(self.h0, P.f('output_layer.2.weight'), P.f('output_layer.2.bias'), self.hh, B, d)
        K.dec_linear(self.hh, P.f('input_layer.0.weight'), self.logits, B, self.V, d, bias=P.f('output_layer.3.bias'))
        # GenerationState.process_logits (generation.py:30-77) on all rows; dead rows are skipped in-kernel
        if st.repetition_penalty > 1.0:
            K.dec_penalty(self.logits, B, None, st.output_ids, self.T, st.cur, st.live_sample_mask,
                          float(st.repetition_penalty))
        K.dec_sample(self.logits, self.V, B, None, st.output_ids, self.T, st.cur, st.live_sample_mask,
                     int(st.end_token), float(st.temperature), int(st.top_k), float(st.top_p), st.seed, st.live_count)
        K.dec_advance(st.cur)

    def run(self, check_every=8):
        """The reference's `while not state.should_stop()` loop (transformer_vae.py:114-126)."""
        st = self.st
        if st.should_stop():
            return st.final_output()
        self._step(first=True)
        st.step_done()
        n = 0
        while st.current_index < self.T - 1:
            if n % check_every == 0 and int(st.live_count.item()) == 0:
                break
            if self.use_graph:
                if self.graph is None:
                    self._capture()
                self.graph.replay()
            else:
                self._step(first=False)
            st.step_done()
            n += 1
        return st.final_output()

    def _capture(self):
        """Capture one generic step. The warm-up/capture launches would advance the device state, so it is
        saved and restored around the capture."""
        st = self.st
        saved = (st.output_ids.clone(), st.live_sample_mask.clone(), st.cur.clone(), st.live_count.clone(),
                 self.kc.clone(), self.vc.clone())
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            self._step(first=False)          # warm-up outside the graph
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._step(first=False)
        st.output_ids.copy_(saved[0])
        st.live_sample_mask.copy_(saved[1])
        st.cur.copy_(saved[2])
        st.live_count.copy_(saved[3])
        self.kc.copy_(saved[4])
        self.vc.copy_(saved[5])
        self.graph = g
