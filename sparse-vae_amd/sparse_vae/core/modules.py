"""Parameter containers with the reference's module tree (so `state_dict` keys match 1:1):
Attention (attention.py:11-49), TransformerLayer (transformer_layer.py:5-42), Perceiver (perceiver.py:5-29),
ConditionalGaussian (conditional_gaussian.py:6-16). Their arithmetic runs in the fused step engine
(sparse_vae/engine.py), not in these modules' forward()."""
import torch
from torch import nn


def _no_forward(name):
    def forward(self, *a, **k):
        raise RuntimeError(f'{name}.forward is not used on MI355X: the step runs in sparse_vae.engine '
                           f'(call TransformerVAE.training_step / reconstruct)')
    return forward


class Attention(nn.Module):
    def __init__(self, d_model, num_heads, causal=False, sparse=False, learned_queries=None, max_length=10000):
        super().__init__()
        assert d_model % num_heads == 0, 'num_heads must divide d_model evenly'    # attention.py:27
        self.causal, self.d_model, self.num_heads, self.max_length = causal, d_model, num_heads, max_length
        if learned_queries:
            self.learned_queries = nn.Parameter(torch.randn(1, learned_queries, d_model))
        else:
            self.q_linear = nn.Linear(d_model, d_model)
            self.learned_queries = None
        self.k_linear = nn.Linear(d_model, d_model)
        self.v_linear = nn.Linear(d_model, d_model)
        self.output_linear = nn.Linear(d_model, d_model)
        self.pos_linear = nn.Linear(d_model, d_model)   # never used by the reference either (no gradient)
        # SparseAttention(window_size=sparse if isinstance(sparse, int) else 4) (attention.py:45-48; note that
        # True is an int there too). Causal sliding window of `window` 32-token blocks plus the [CLS] block,
        # rotary base 2 * window * 32 (attention.py:52); run by the attention kernel's window mode.
        self.sparse_window = (int(sparse) if isinstance(sparse, int) else 4) if sparse else 0
        if self.sparse_window and not causal:
            raise NotImplementedError('non-causal sparse attention (two-sided window) is not used by the reference')

    forward = _no_forward('Attention')


class TransformerLayer(nn.Module):
    def __init__(self, d_model, num_heads, causal=False, use_cross_attention=False, sparse_self_attention=False,
                 learned_queries=None):
        super().__init__()
        self.attention = Attention(d_model, num_heads, causal, learned_queries=learned_queries,
                                   sparse=sparse_self_attention)
        self.ffn = nn.Sequential(nn.Linear(d_model, d_model * 4), nn.GELU(), nn.Linear(d_model * 4, d_model, bias=False))
        self.dropout = nn.Dropout(p=0.1)
        self.attn_layer_norm = nn.LayerNorm(d_model)
        self.ffn_layer_norm = nn.LayerNorm(d_model)
        if use_cross_attention:
            self.cross_attention = Attention(d_model, num_heads)
            self.cross_attn_layer_norm = nn.LayerNorm(d_model)
            self.context_layer_norm = nn.LayerNorm(d_model)
        else:
            self.cross_attention = None

    @property
    def use_cross_attention(self):
        return self.cross_attention is not None

    forward = _no_forward('TransformerLayer')


class Perceiver(nn.Module):
    def __init__(self, num_layers, num_latents, d_model, bottleneck_width=None, self_attention_layers=1):
        super().__init__()
        assert num_layers > 1                                                      # perceiver.py:12
        num_heads = d_model // 64                                                  # perceiver.py:13
        self.first_layer = TransformerLayer(d_model, num_heads, learned_queries=num_latents)
        if bottleneck_width:
            self.bottleneck = TransformerLayer(d_model, num_heads, learned_queries=bottleneck_width)
            num_layers -= 1
        else:
            self.bottleneck = None
        self.middle_layers = nn.ModuleList([TransformerLayer(d_model, num_heads, use_cross_attention=True)
                                            for _ in range(num_layers - 1)])

    forward = _no_forward('Perceiver')


class ConditionalGaussian(nn.Module):
    def __init__(self, in_features, out_features, zero_initialized=False, bias=True):
        super().__init__()
        self.linear = nn.Linear(in_features, out_features * 2, bias=bias)
        if zero_initialized:
            with torch.no_grad():
                self.linear.weight.zero_()
                if bias:
                    self.linear.bias.zero_()

    forward = _no_forward('ConditionalGaussian')
