"""sparse-vae on MI355X: the TransformerVAE training hot path of norabelrose/sparse-vae on hand-written gfx950
kernels (libsvae.so, C ABI in include/svae.h), behind the reference's Python surface."""
from .core import *  # noqa: F401,F403
from .core import PaddedTensor, RAdam, marginal_kl  # noqa: F401
from .transformer_vae import TransformerVAE, TransformerVAEHparams  # noqa: F401
from .text_data_module import TextDataModule  # noqa: F401
from .trainer import Trainer, seed_everything  # noqa: F401
from .core.auto_select_gpu import select_best_gpu  # noqa: F401
