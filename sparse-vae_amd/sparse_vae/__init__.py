"""sparse-vae on MI355X: the TransformerVAE training hot path on hand-written gfx950 kernels (libsvae.so)."""
