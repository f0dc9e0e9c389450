"""ORACLE — test infrastructure only.

This package is a CPU fp32 restatement of the reference TransformerVAE training step
(norabelrose/sparse-vae, `sparse_vae/transformer_vae.py:42-66` and the modules it calls).
It exists to CHECK the HIP product path; it is never shipped or measured as the product.

Only `tests/`, `__graft_entry__.smoke()` and the `cpu_baseline` leg of `bench.py` may import it.
The product package (`sparse-vae_amd/sparse_vae`) never imports anything from here and fails
loudly when its HIP library is missing.

Pinning: `tests/golden/make_golden.py` imports the real reference in the survey container
(through stubs for the absent third-party modules) and writes golden vectors to
`tests/golden/*.npz`; `tests/test_oracle_golden.py` checks this restatement against them.
"""
from .params import param_shapes, init_params, HParams  # noqa: F401
from .svae_oracle import *  # noqa: F401,F403
