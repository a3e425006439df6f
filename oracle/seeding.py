"""Deterministic weight / input generators shared by the golden-fixture script,
the CPU oracle and the parity tests.

TEST INFRASTRUCTURE ONLY: imported by tests/, bench.py's cpu_baseline leg,
__graft_entry__.smoke() and tests/golden/make_golden.py. Never by the product.

Weights are generated per state_dict key from a generator seeded by
crc32(key) ^ seed, so any module whose state_dict has the reference's key
names (models.py:183-403) receives identical values regardless of the order
in which its parameters were constructed.  Every zero-initialised branch of
the reference (``gamma`` at models.py:101,138,275 and the affine heads'
linear2 at models.py:63-67) is given non-zero values so all paths are live.
"""
import zlib

import numpy as np
import torch


def _gen(key, seed):
    g = torch.Generator()
    g.manual_seed((zlib.crc32(key.encode()) ^ (seed * 2654435761)) & 0x7FFFFFFF)
    return g


def seeded_value(key, shape, seed=0, dtype=torch.float32):
    """One state_dict entry. The value distribution depends only on the key's
    role (weight / bias / BN affine / running stats / residual gamma)."""
    shape = tuple(int(s) for s in shape)
    g = _gen(key, seed)
    leaf = key.rsplit('.', 1)[-1]
    if leaf == 'num_batches_tracked':
        return torch.zeros(shape, dtype=torch.long)
    if leaf == 'running_mean':
        return (torch.randn(shape, generator=g) * 0.1).to(dtype)
    if leaf == 'running_var':
        return (torch.rand(shape, generator=g) + 0.5).to(dtype)
    if leaf == 'gamma' and shape == (1,):
        return (0.5 + 0.2 * torch.rand(shape, generator=g)).to(dtype)
    if len(shape) >= 2:
        fan_in = int(np.prod(shape[1:]))
        return (torch.randn(shape, generator=g) / np.sqrt(fan_in)).to(dtype)
    # 1-D
    if leaf == 'weight':  # BN affine weight
        return (1.0 + 0.1 * torch.randn(shape, generator=g)).to(dtype)
    return (0.1 * torch.randn(shape, generator=g)).to(dtype)


def seeded_state(spec, seed=0):
    """spec: iterable of (key, shape) -> OrderedDict of tensors."""
    from collections import OrderedDict
    return OrderedDict((k, seeded_value(k, s, seed)) for k, s in spec)


def state_spec(state_dict):
    return [(k, tuple(v.shape)) for k, v in state_dict.items()]


def seeded_tensor(name, shape, seed=0, kind='normal', lo=-1.0, hi=1.0):
    g = _gen('input:' + name, seed)
    if kind == 'normal':
        return torch.randn(tuple(shape), generator=g)
    if kind == 'uniform':
        return torch.rand(tuple(shape), generator=g) * (hi - lo) + lo
    raise ValueError(kind)


def seeded_ints(name, shape, lo, hi, seed=0):
    """Integers uniform in [lo, hi] inclusive, int64."""
    g = _gen('int:' + name, seed)
    return torch.randint(lo, hi + 1, tuple(shape), generator=g, dtype=torch.long)


def synthetic_batch(B, seed=3407, n_words=5450, words_num=20, class_num=200,
                    attr_num=3, attr_len=5, sizes=(64, 128, 256), emb_dim=256):
    """The bench/test synthetic batch: images U(-1,1) at 3
    scales, captions int64 (B,20) tokens U[1,n_words) with lengths U[5,18],
    zero padded, attributes (B,3,5) with lengths U[1,5], unpaired captions,
    class ids U[1,class_num]."""
    imgs = [seeded_tensor('img%d' % s, (B, 3, s, s), seed, 'uniform') for s in sizes]
    cap_lens = seeded_ints('cap_lens', (B,), 5, 18, seed)
    caps = seeded_ints('caps', (B, words_num), 1, n_words - 1, seed)
    caps = caps * (torch.arange(words_num)[None, :] < cap_lens[:, None]).long()
    attrs_len = seeded_ints('attrs_len', (B, attr_num), 1, attr_len, seed)
    attrs = seeded_ints('attrs', (B, attr_num, attr_len), 1, n_words - 1, seed)
    attrs = attrs * (torch.arange(attr_len)[None, None, :] < attrs_len[..., None]).long()
    un_lens = seeded_ints('unpair_cap_lens', (B,), 5, 18, seed)
    un_caps = seeded_ints('unpair_caps', (B, words_num), 1, n_words - 1, seed)
    un_caps = un_caps * (torch.arange(words_num)[None, :] < un_lens[:, None]).long()
    cls_ids = seeded_ints('cls_ids', (B,), 1, class_num, seed)
    noise = seeded_tensor('noise', (B, 100), seed)
    return dict(imgs=imgs, caps=caps, cap_lens=cap_lens, attrs=attrs, attrs_len=attrs_len,
                unpair_caps=un_caps, unpair_cap_lens=un_lens, cls_ids=cls_ids, noise=noise)


def summary(t, n_samples=512):
    """Size-independent fingerprint of a tensor: full values when small,
    else [numel, sum, abs-sum, sq-sum, max, min] + values at fixed indices."""
    t = t.detach().double().reshape(-1).cpu()
    n = t.numel()
    if n <= 4096:
        return t.numpy().copy()
    g = torch.Generator()
    g.manual_seed(n)
    idx = torch.randperm(n, generator=g)[:n_samples]
    head = torch.tensor([n, t.sum().item(), t.abs().sum().item(), (t * t).sum().item(),
                         t.max().item(), t.min().item()], dtype=torch.float64)
    return torch.cat([head, t[idx]]).numpy()


def compare_summary(a, b, rtol, atol):
    """Compare two summaries (numpy). Returns (ok, max_abs_err, info)."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    if a.shape != b.shape:
        return False, float('inf'), 'shape %s vs %s' % (a.shape, b.shape)
    err = np.abs(a - b)
    tol = atol + rtol * np.abs(b)
    bad = err > tol
    return (not bad.any()), float(err.max() if err.size else 0.0), int(bad.sum())
