"""Configuration tree with the reference's keys and defaults
(miscc/config.py:9-67) and a YAML loader that merges a file into it with the
same key/type checking (miscc/config.py:69-108).

Differences from the reference, both deliberate: the YAML is read with
yaml.safe_load (the reference's bare yaml.load fails on PyYAML >= 6), and the
keys GPU_ID used by cfg/coco.yml and cfg/flower.yml are accepted."""
import numpy as np


class AttrDict(dict):
    """dict with attribute access (what the reference gets from easydict)."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError:
            raise AttributeError(k)

    def __setattr__(self, k, v):
        self[k] = AttrDict(v) if (isinstance(v, dict) and not isinstance(v, AttrDict)) else v


def _tree(d):
    out = AttrDict()
    for k, v in d.items():
        out[k] = _tree(v) if isinstance(v, dict) else v
    return out


cfg = _tree({
    'DATASET_NAME': 'bird', 'CONFIG_NAME': '', 'DATA_DIR': '', 'SAVE_DIR': '', 'WORKERS': 4,
    'RNN_TYPE': 'LSTM', 'CUDA': True, 'GPU_ID': 0,
    'TREE': {'BRANCH_NUM': 3, 'BASE_SIZE': 64},
    'TRAIN': {
        'USE_ATTR': True, 'USE_UNPAIR': True, 'USE_CLASS': True, 'CLASS_NUM': 200,
        'NET_E': '', 'NET_G': '', 'BATCH_SIZE': 64, 'MAX_EPOCH': 600, 'WARMUP_EPOCHS': 200,
        'GSAVE_INTERVAL': 10, 'DSAVE_INTERVAL': 10,
        'DISCRIMINATOR_LR': 2e-4, 'GENERATOR_LR': 2e-4, 'ENCODER_LR': 2e-4, 'RNN_GRAD_CLIP': 0.25,
        'SMOOTH': {'GAMMA1': 5.0, 'GAMMA3': 10.0, 'GAMMA2': 5.0, 'LAMBDA': 1.0},
    },
    'GAN': {'GF_DIM': 64, 'DF_DIM': 64, 'Z_DIM': 100, 'CONDITION_DIM': 100},
    'TEXT': {'MAX_ATTR_NUM': 3, 'MAX_ATTR_LEN': 5, 'CAPTIONS_PER_IMAGE': 10, 'EMBEDDING_DIM': 256,
             'WORDS_NUM': 20, 'DAMSM_NAME': ''},
})
__C = cfg


def _merge(src, dst, path=''):
    for k, v in src.items():
        if k not in dst:
            raise KeyError('{} is not a valid config key'.format(path + k))
        old = dst[k]
        if isinstance(old, dict):
            if not isinstance(v, dict):
                raise ValueError('Type mismatch for config key: {}'.format(path + k))
            _merge(v, old, path + k + '.')
            continue
        if type(old) is not type(v):
            if isinstance(old, np.ndarray):
                v = np.array(v, dtype=old.dtype)
            elif isinstance(old, float) and isinstance(v, int):
                v = float(v)
            else:
                raise ValueError('Type mismatch ({} vs. {}) for config key: {}'.format(type(old), type(v), path + k))
        dst[k] = v


def cfg_from_file(filename):
    import yaml
    with open(filename, 'r') as f:
        _merge(yaml.safe_load(f) or {}, cfg)
