"""TransformerHparams and VOCAB_SIZE (transformer_language_model.py:13-30 in the reference)."""
from dataclasses import dataclass
from typing import Optional

from .language_model import LanguageModelHparams

VOCAB_SIZE = 2 ** 15   # transformer_language_model.py:13


@dataclass
class TransformerHparams(LanguageModelHparams):
    d_embedding: Optional[int] = None
    d_model: int = 512
    num_heads: int = 8
    num_layers: int = 6
    input_dropout: float = 0.0
    tie_embedding_weights: bool = True
    cross_attention: bool = False
    grad_checkpointing: bool = False
    separate_context_embedding: bool = True
    attn_window_size: int = 4
    sparse_self_attention: bool = True
