"""CPU tests: the C-ABI library loads and exports every symbol include/eegan_hip.h
declares; the drop-in modules expose the reference's state_dict keys and
shapes (so reference checkpoints load); config parsing; host logic."""
import os
import re

import pytest
import torch

from _util import REPO, spec


def test_library_exports_header_symbols():
    import eegan_hip
    from eegan_hip import _lib
    hdr = open(os.path.join(REPO, 'include', 'eegan_hip.h')).read()
    declared = sorted(set(re.findall(r'\b(eegan_[a-z0-9_]+)\s*\(', hdr)))
    assert len(declared) >= 60
    for name in declared:
        assert hasattr(_lib.LIB, name), name          # exported by libeegan_hip.so
        assert name in _lib._SIGS, name               # bound with a ctypes signature
    assert set(_lib._SIGS) == set(declared)
    assert eegan_hip.ABI_VERSION == 17
    # rows padded to 128; every tap's channel run padded to 32 (to 8 for <= 8
    # channels: 4 taps per K step), rows padded to whole 32-deep steps
    assert _lib.ops.conv_packed_elems(100, 3, 3, 3, 0) == 128 * 96
    assert _lib.ops.conv_packed_elems(100, 3, 3, 3, 1) == 128 * 9 * 128
    assert _lib.ops.conv_packed_elems(3, 32, 3, 3, 1) == 128 * 96
    assert _lib.ops.conv_packed_elems(64, 48, 4, 4, 0) == 128 * 16 * 64
    from eegan_hip.tensor import ld_for
    assert ld_for(3) == 8 and ld_for(100) == 104 and ld_for(1, torch.float32) == 1


def _keys(mod):
    return [(k, tuple(v.shape)) for k, v in mod.state_dict().items()]


def test_state_dict_parity_with_reference():
    import models
    import DAMSM
    from sync_batchnorm import SynchronizedBatchNorm2d
    cases = [
        ('gen', models.Gen(8, 100)),
        ('sagb_sc', models.SAGB_Block(16, 8, pred_mask=True)),
        ('sagb_id', models.SAGB_Block(16, 16, pred_mask=True)),
        ('sagb_nomask', models.SAGB_Block(8, 8, pred_mask=False)),
        ('cum', models.Cum_Block(16, 8)),
        ('resd_sc', models.resD(8, 16)),
        ('resd_id', models.resD(16, 16)),
        ('discsent', models.DiscSent(32, 256)),
        ('disccond', models.DiscCond(32, 256, class_nums=10)),
        ('attr', models.ATTR_Enhance()),
        ('syncbn', SynchronizedBatchNorm2d(8)),
        ('dis64', models.Dis64(8)),
        ('dis128', models.Dis128(8)),
        ('dis256', models.Dis256(8, True, 10)),
        ('rnn', DAMSM.RNN_ENCODER(50, nhidden=256)),
    ]
    for name, mod in cases:
        assert _keys(mod) == spec(name), name


def test_dataparallel_prefix_and_module():
    import models
    from sync_batchnorm import DataParallelWithCallback
    g = DataParallelWithCallback(models.Gen(8, 100))
    keys = list(g.state_dict().keys())
    assert len(keys) == 262 and all(k.startswith('module.') for k in keys)
    assert 'module.blocks.0.affine1.norm2d.running_mean' in keys
    assert isinstance(g.module, models.Gen)


def test_cnn_encoder_keys_torchvision_names():
    import DAMSM
    enc = DAMSM.CNN_ENCODER(256)
    sd = enc.state_dict()
    for k in ['Conv2d_1a_3x3.conv.weight', 'Conv2d_1a_3x3.bn.running_var', 'Mixed_5b.branch_pool.conv.weight',
              'Mixed_6e.branch7x7dbl_5.conv.weight', 'Mixed_7c.branch3x3dbl_3b.bn.bias', 'emb_features.weight',
              'emb_cnn_code.bias']:
        assert k in sd, k
    assert tuple(sd['Mixed_6b.branch7x7_2.conv.weight'].shape) == (128, 128, 1, 7)
    assert tuple(sd['emb_cnn_code.weight'].shape) == (256, 2048)
    assert not any(p.requires_grad for p in enc.parameters())


def test_config_merge(tmp_path):
    from miscc.config import cfg, cfg_from_file
    y = tmp_path / 'bird.yml'
    y.write_text('CONFIG_NAME: x\nDATASET_NAME: bird\nGPU_ID: 0\nTRAIN:\n  BATCH_SIZE: 16\n  CLASS_NUM: 200\n'
                 'GAN:\n  GF_DIM: 32\n  DF_DIM: 32\n')
    old = (cfg.TRAIN.BATCH_SIZE, cfg.GAN.GF_DIM, cfg.GAN.DF_DIM)
    cfg_from_file(str(y))
    assert cfg.TRAIN.BATCH_SIZE == 16 and cfg.GAN.GF_DIM == 32 and cfg.TRAIN.SMOOTH.GAMMA1 == 5.0
    bad = tmp_path / 'bad.yml'
    bad.write_text('NOT_A_KEY: 1\n')
    with pytest.raises(KeyError):
        cfg_from_file(str(bad))
    cfg.TRAIN.BATCH_SIZE, cfg.GAN.GF_DIM, cfg.GAN.DF_DIM = old


def test_att_maps_lazy_list():
    from miscc.DAMSM_losses import _AttMaps
    att = torch.arange(2 * 3 * 289, dtype=torch.float32).reshape(2, 3, 289)
    m = _AttMaps(att, torch.tensor([3, 1]))
    assert len(m) == 2 and m[1].shape == (1, 1, 17, 17) and m[0].shape == (1, 3, 17, 17)


def test_early_term_roots_match_joint_backward():
    """g_update's backward from per-D terms already differentiated at their
    (aliased) fake images (trainer.EarlyTerm, EEGAN_GTERM_GRAD_EARLY) gives the
    generator the same gradients as backward of the summed loss (train.py:
    477-493: g_loss is linear in the terms)."""
    from eegan_hip.trainer import EarlyTerm, _backward_roots, _term_value
    torch.manual_seed(0)
    w = torch.nn.Parameter(torch.randn(4, 4, dtype=torch.float64))
    z = torch.randn(3, 4, dtype=torch.float64)
    d = [torch.randn(4, 4, dtype=torch.float64) for _ in range(2)]

    def fakes():
        h = torch.tanh(z @ w)
        return [h, torch.sin(h @ w)]            # two "stages" sharing w

    def term(i, img):
        return (torch.tanh(img @ d[i]) ** 2).sum()

    f = fakes()
    (ref,) = torch.autograd.grad(term(0, f[0]) + term(1, f[1]), w)
    f = fakes()
    terms = []
    for i in range(2):
        alias = f[i].view_as(f[i])
        t = term(i, alias)
        (g,) = torch.autograd.grad(t, alias)
        terms.append(EarlyTerm(t.detach(), alias, g))
    roots, grads = _backward_roots(terms)
    (got,) = torch.autograd.grad(roots, w, grads)
    assert torch.allclose(got, ref, rtol=1e-12, atol=1e-12)
    assert float(_term_value(terms[0]) + _term_value(terms[1])) == pytest.approx(
        float(term(0, f[0]) + term(1, f[1])))


def test_words_loss_refuses_wide_captions():
    """words_loss with captions wider than the kernel's 32 words raises a
    clear error before any device work (no silent truncation)."""
    import torch
    from eegan_hip.functional import WordsSimFn
    regions = torch.zeros(2, 256, 17, 17)
    words = torch.zeros(2, 256, 33)
    with pytest.raises(ValueError, match='up to 32 words'):
        WordsSimFn.apply(regions, words, torch.tensor([33, 5]), False, 0)


def test_gradient_penalty_mask_sources_detached_only_inside_the_scope():
    """functional._mask_src: an act' mask's source activation is detached only
    inside detached_mask_sources (Trainer.MA_gradient_penalty's first backward)
    and only for piecewise-constant activations (none / relu / leaky relu); a
    tanh / sigmoid source keeps its graph (its second derivative is not zero),
    and the flag is restored on exit, also after an exception."""
    import torch
    from eegan_hip import functional as Fn
    from eegan_hip._lib import ACT_CODES
    t = torch.ones(3, requires_grad=True) * 2.0
    assert Fn._mask_src(t, ACT_CODES['lrelu']) is t
    with Fn.detached_mask_sources():
        for act in ('relu', 'lrelu', 'none'):
            d = Fn._mask_src(t, ACT_CODES[act])
            assert not d.requires_grad and d.data_ptr() == t.data_ptr()
        for act in ('tanh', 'sigmoid'):
            assert Fn._mask_src(t, ACT_CODES[act]) is t
        assert Fn._mask_src(None, ACT_CODES['relu']) is None
    assert not Fn.DETACH_MASK_SRC
    try:
        with Fn.detached_mask_sources():
            raise KeyError('x')
    except KeyError:
        pass
    assert not Fn.DETACH_MASK_SRC
    with Fn.detached_mask_sources(False):
        assert Fn._mask_src(t, ACT_CODES['relu']) is t


def test_replication_callbacks_one_process():
    """sync_batchnorm.replicate's callback API (replicate.py:23-88) in one
    process: wrapping runs __data_parallel_replicate__ on every SyncBN with
    copy_id = the rank (0), one shared context per submodule position whose
    sync_master is the rank group; a single copy is not parallel (the
    reference keeps F.batch_norm then, batchnorm.py:50)."""
    import models
    from sync_batchnorm import (CallbackContext, DataParallelWithCallback, execute_replication_callbacks,
                                patch_replication_callback)
    g = DataParallelWithCallback(models.Gen(8, 100))
    bns = [m for m in g.module.modules() if hasattr(m, '__data_parallel_replicate__')]
    assert bns and all(m._parallel_id == 0 and not m._is_parallel for m in bns)
    assert all(m._sync_group.world == 1 and m._sync_group.rank == 0 for m in bns)
    assert g.replicate(g.module, [0]) == [g.module]
    # two copies in one process (the reference's own replicate): master first, shared contexts
    seen = []

    class M(torch.nn.Module):
        def __data_parallel_replicate__(self, ctx, copy_id):
            seen.append((id(ctx), copy_id))
    a, b = torch.nn.Sequential(M()), torch.nn.Sequential(M())
    ctxs = execute_replication_callbacks([b, a], copy_ids=[1, 0])
    assert [c for _, c in seen] == [0, 1] and seen[0][0] == seen[1][0]
    assert isinstance(ctxs[1], CallbackContext) and ctxs[1].sync_master.world == 1
    dp = torch.nn.DataParallel(models.ATTR_Enhance())
    assert patch_replication_callback(dp) is dp
