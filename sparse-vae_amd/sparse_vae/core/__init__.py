from .padded_tensor import PaddedTensor
from .language_model import LanguageModel, LanguageModelHparams, AttributeDict, cosine_decay
from .transformer_language_model import TransformerHparams, VOCAB_SIZE
from .continuous_autoencoder import ContinuousVAEHparams, ContinuousVAEHooks
from .modules import Attention, TransformerLayer, Perceiver, ConditionalGaussian
from .rectified_adam import RAdam
from .math_utils import marginal_kl
