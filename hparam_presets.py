"""Named presets for `python train.py transformer-vae preset=NAME` (hparam_presets.py in the reference), plus
the build's own: 'tiny' (smallest buildable model: Perceiver needs num_layers // 2 > 1) and the benchmark
configs of BASELINE.json. All model presets here use the dense attention path."""

_wiki = dict(dataset_name='wikipedia', dataset_config='20200501.en')

hparam_presets = {
    # -------- build-defined (synthetic data, BASELINE.json configs)
    'tiny': {
        'data': dict(dataset_name='synthetic', seq_len=128, batch_size=64),
        'model': dict(d_model=128, num_layers=4, num_heads=8, latent_depth=64, sparse_self_attention=False,
                      grad_clip_threshold=150.0, init_scale=0.02, lr=3e-4),
        'trainer': dict(accumulate_grad_batches=1),
    },
    'c2': {   # 6 layers, d_model 512, seq 512, batch 64 per GPU
        'data': dict(dataset_name='synthetic', seq_len=512, batch_size=64),
        'model': dict(d_model=512, num_layers=6, num_heads=8, latent_depth=64, sparse_self_attention=False,
                      grad_clip_threshold=150.0, init_scale=0.02, kl_weight_start=0.3, kl_weight_end=1.0,
                      kl_annealing_steps=8000, lr=3e-4),
        'trainer': dict(accumulate_grad_batches=1),
    },
    'c4': {   # 12 layers, d_model 768, seq 1024, 64 per GPU (global 512 on 8 GPUs)
        'data': dict(dataset_name='synthetic', seq_len=1024, batch_size=64),
        'model': dict(d_model=768, num_layers=12, num_heads=8, latent_depth=64, sparse_self_attention=False,
                      grad_clip_threshold=150.0, init_scale=0.02, lr=3e-4),
        'trainer': dict(accumulate_grad_batches=1),
    },
    'c5': {   # the C4 model at seq 2048
        'data': dict(dataset_name='synthetic', seq_len=2048, batch_size=32),
        'model': dict(d_model=768, num_layers=12, num_heads=8, latent_depth=64, sparse_self_attention=False,
                      grad_clip_threshold=150.0, init_scale=0.02, lr=3e-4),
        'trainer': dict(accumulate_grad_batches=1),
    },
    # -------- the reference's presets (hparam_presets.py:1-202); real-data paths need dataset_path offline
    'dense-benchmark': {
        'data': dict(**_wiki, tokens_per_batch=50_000, min_tokens_per_sample=512, max_tokens_per_sample=3_125),
        'model': dict(d_model=512, grad_checkpointing=True, grad_clip_threshold=150.0, init_scale=0.02,
                      kl_weight_start=0.3, kl_weight_end=1.0, kl_annealing_steps=8000, latent_depth=64, lr=3e-4,
                      num_layers=6, sparse_self_attention=False, tie_embedding_weights=True),
        'trainer': dict(accumulate_grad_batches=2),
    },
    'sparse-benchmark': {
        'data': dict(**_wiki, tokens_per_batch=50_000, min_tokens_per_sample=512, max_tokens_per_sample=3_125),
        'model': dict(d_model=512, grad_checkpointing=True, grad_clip_threshold=150.0, init_scale=0.02,
                      kl_weight_start=1.0, kl_annealing_steps=0, latent_depth=64, lr=3e-4, num_layers=6,
                      sparse_self_attention=True, tie_embedding_weights=True),
        'trainer': dict(accumulate_grad_batches=2),
    },
    'wikipedia': {
        'data': dict(**_wiki, tokens_per_batch=100_000, min_tokens_per_sample=512, max_tokens_per_sample=50_000),
        'model': dict(d_model=512, grad_checkpointing=True, grad_clip_threshold=150.0, init_scale=0.02,
                      attn_window_size=8, kl_weight_start=0.1, kl_weight_end=1.0, kl_annealing_steps=8000,
                      latent_depth=64, lr=3e-4, num_layers=6, sparse_self_attention=True, tie_embedding_weights=True),
        'trainer': dict(accumulate_grad_batches=2, val_check_interval=0.1),
    },
    'pg19': {
        'data': dict(dataset_name='pg19', dataset_config=None, tokens_per_batch=102_912, min_tokens_per_sample=512,
                     max_tokens_per_sample=102_400),
        'model': dict(d_model=512, grad_checkpointing=True, grad_clip_threshold=150.0, init_scale=0.02,
                      attn_window_size=6, kl_weight_start=0.1, kl_weight_end=1.0, kl_annealing_steps=8000,
                      latent_depth=64, lr=3e-4, num_layers=6, sparse_self_attention=True, tie_embedding_weights=True),
        'trainer': dict(accumulate_grad_batches=4, val_check_interval=0.5),
    },
}
