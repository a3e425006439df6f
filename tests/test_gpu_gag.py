"""GlobalAttentionGeneral on the GPU (csrc/gag.hip via miscc.DAMSM_losses)
against the golden vectors captured from the reference
(DAMSM_losses.py:65-132: damsm/gag_wc, damsm/gag_att, which include the
reference's mask.repeat(queryL, 1) row indexing) and against the fp32 oracle's
autograd for the backward, for source lengths within one 64-source chunk and
across several (100, 300: the online-softmax path).

Tolerances: the logits and the weighted context are split-bf16 MFMA products
(hi*hi + lo*hi + hi*lo, relative error per product ~2^-16), so the forward is
gated at 1e-4 of the output's max magnitude; the backward (fp32 SIMT from the
saved attention) at rel-L2 1e-4."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from _util import golden, rel_l2  # noqa: E402
from oracle.seeding import seeded_tensor  # noqa: E402

TOL_GAG_FWD = 1e-4
TOL_GAG_BWD = 1e-4


def _module(mask):
    from miscc.DAMSM_losses import GlobalAttentionGeneral
    m = GlobalAttentionGeneral(32, 32)
    if mask is not None:
        m.applyMask(mask)
    return m


def test_gag_golden(gpu):
    g = golden()
    inp = seeded_tensor('dm:gin', (2, 32, 6, 6), 1)
    key = seeded_tensor('dm:gkey', (2, 32, 9), 1)
    val = seeded_tensor('dm:gval', (2, 32, 9), 1)
    gmask = torch.zeros(2, 9, dtype=torch.bool)
    gmask[0, 7:] = True
    gmask[1, 4:] = True
    wc, att = _module(gmask.to(gpu))(inp.to(gpu), key.to(gpu), val.to(gpu))
    for name, got in (('gag_wc', wc), ('gag_att', att)):
        ref = np.asarray(g['damsm/' + name], np.float64).reshape(-1)
        got = got.detach().double().cpu().numpy().reshape(-1)
        assert got.shape == ref.shape
        err = np.abs(got - ref).max()
        assert err <= TOL_GAG_FWD * np.abs(ref).max(), (name, err)


@pytest.mark.parametrize('B,idf,cdf,ih,iw,S,masked', [
    (3, 48, 40, 20, 20, 37, True),   # 7 query tiles (ragged last), ragged idf / cdf K-steps
    (1, 7, 3, 1, 5, 64, False),      # queryL < one tile, sourceL at the maximum, tiny channels
    (4, 256, 32, 17, 17, 18, True),  # DAMSM-like shapes: 289 regions x 18 words
    (2, 64, 96, 9, 11, 100, True),   # sources beyond one 64-chunk: 2 chunks, 2 channel groups
    (2, 40, 24, 5, 7, 300, True),    # 5 chunks, ragged last chunk, masked tails
    (1, 16, 8, 3, 3, 300, False),
])
def test_gag_fwd_bwd(gpu, B, idf, cdf, ih, iw, S, masked):
    from oracle import eegan_oracle as O
    torch.manual_seed(B * 1000 + S)
    inp = torch.randn(B, idf, ih, iw) * 0.3
    key = torch.randn(B, idf, S) * 0.3
    val = torch.randn(B, cdf, S)
    mask = None
    if masked:  # ragged per-row lengths, never a fully masked row
        lens = torch.randint(1, S + 1, (B,))
        mask = torch.arange(S)[None, :] >= lens[:, None]
    gw = torch.randn(B, cdf, ih, iw)
    ga = torch.randn(B, S, ih, iw)
    xr, kr, vr = (t.clone().requires_grad_() for t in (inp, key, val))
    wcr, attr = O.global_attention_general(xr, kr, vr, mask)
    ((wcr * gw).sum() + (attr * ga).sum()).backward()
    outs = []
    for _ in range(2):
        x, k, v = (t.to(gpu).requires_grad_() for t in (inp, key, val))
        wc, att = _module(mask.to(gpu) if mask is not None else None)(x, k, v)
        ((wc * gw.to(gpu)).sum() + (att * ga.to(gpu)).sum()).backward()
        outs.append([t.detach().cpu() for t in (wc, att, x.grad, k.grad, v.grad)])
    wc, att, dx, dk, dv = outs[0]
    assert wc.shape == wcr.shape and att.shape == attr.shape
    assert (wc - wcr.detach()).abs().max() <= TOL_GAG_FWD * wcr.detach().abs().max()
    assert (att - attr.detach()).abs().max() <= TOL_GAG_FWD
    if mask is not None:  # masked sources get exactly zero attention
        rows = (torch.arange(B * ih * iw) % B).reshape(B, 1, ih * iw)
        m = mask[rows.expand(B, S, ih * iw), torch.arange(S)[None, :, None].expand(B, S, ih * iw)]
        assert (att.reshape(B, S, -1)[m] == 0).all()
    for name, got, ref in (('dinput', dx, xr.grad), ('dkey', dk, kr.grad), ('dvalue', dv, vr.grad)):
        assert rel_l2(got, ref) <= TOL_GAG_BWD, (name, rel_l2(got, ref))
    for a, b in zip(outs[0], outs[1]):  # deterministic (no atomics)
        assert torch.equal(a, b)


def test_gag_fully_masked_row_is_nan_like_the_reference(gpu):
    """A row whose sources are all masked: the reference's softmax of an
    all -inf row gives NaN (DAMSM_losses.py:121-122); so does the kernel."""
    x = torch.randn(1, 8, 2, 2, device=gpu)
    key, val = torch.randn(1, 8, 70, device=gpu), torch.randn(1, 4, 70, device=gpu)
    wc, att = _module(torch.ones(1, 70, dtype=torch.bool, device=gpu))(x, key, val)
    assert torch.isnan(att).all() and torch.isnan(wc).all()
