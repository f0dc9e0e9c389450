"""python train.py transformer-vae [section.key=value ...] [preset=NAME]

Drop-in for the reference CLI (train.py:12-95): same model name, OmegaConf-style dotlist (model.*, data.*,
trainer.*) and named presets merged AFTER the dotlist (train.py:57-61, so a preset overrides the command
line, as in the reference). OmegaConf / Lightning are not installed here: the dotlist is parsed directly
and the fit loop is sparse_vae.Trainer. Multi-GPU: python -m torch.distributed.run --nproc-per-node N
--master-addr 127.0.0.1 train.py ... (one process per GPU, RCCL data parallelism).
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), 'sparse-vae_amd'))

import yaml  # noqa: E402

from hparam_presets import hparam_presets  # noqa: E402


def parse_dotlist(args):
    cfg = {}
    for a in args:
        if '=' not in a:
            raise SystemExit(f"expected key=value, got '{a}'")
        key, val = a.split('=', 1)
        val = yaml.safe_load(val) if val != '' else None
        node = cfg
        parts = key.split('.')
        for p in parts[:-1]:
            node = node.setdefault(p, {})
        node[parts[-1]] = val
    return cfg


def merge(dst, src):
    for k, v in src.items():
        if isinstance(v, dict) and isinstance(dst.get(k), dict):
            merge(dst[k], v)
        else:
            dst[k] = v
    return dst


def build_config(argv):
    config = {'trainer': {'accumulate_grad_batches': 2}, 'model': {}, 'data': {}}   # train.py:16-23
    merge(config, parse_dotlist(argv))
    preset = config.get('preset')
    if preset:
        preset_config = hparam_presets.get(preset)
        assert preset_config, f"Preset name '{preset}' not recognized."
        merge(config, preset_config)
    return config


def main(args):
    if len(args) < 2:
        raise SystemExit(__doc__)
    model_str = args[1]
    from sparse_vae import TransformerVAE, TransformerVAEHparams, TextDataModule, Trainer, seed_everything
    seed_everything(7295)                                                            # train.py:15
    if model_str != 'transformer-vae':
        print(f"Model type '{model_str}' is not on the MI355X path (only 'transformer-vae' is).")
        raise SystemExit(1)
    config = build_config(args[2:])
    hparams = TransformerVAEHparams(**config['model'])
    print('Training transformer-vae...')
    model = TransformerVAE(hparams)
    data = TextDataModule(**config.get('data', {}))
    trainer = Trainer(**config['trainer'])
    trainer.fit(model, datamodule=data)
    return trainer


if __name__ == '__main__':
    main(sys.argv)
