"""Pin the CPU oracle (oracle/eegan_oracle.py) to golden vectors captured by
importing the reference on CPU (tests/golden/make_golden.py)."""
import json

import numpy as np
import pytest
import torch

from _util import golden, golden_state, assert_close_fp, fp
from oracle import eegan_oracle as O
from oracle.seeding import seeded_tensor, seeded_ints, seeded_state, synthetic_batch

RT, AT = 2e-4, 2e-5


def _req(sd):
    for k, v in sd.items():
        if v.is_floating_point() and 'running' not in k:
            v.requires_grad_(True)
    return sd


def _check_grads(tag, sd, rt=RT, at=AT):
    g = golden()
    n = 0
    for k, v in sd.items():
        key = tag + '/grad/' + k
        if key in g:
            assert v.grad is not None, key
            assert_close_fp(key, fp(v.grad), g[key], rt, at)
            n += 1
    assert n > 0


@pytest.mark.parametrize('tag,cin,cout,pm,res', [('sagb_sc', 16, 8, True, 8), ('sagb_id', 16, 16, True, 4),
                                                 ('sagb_nomask', 8, 8, False, 8)])
def test_sagb_block(tag, cin, cout, pm, res):
    g = golden()
    sd = _req(golden_state(tag, 11))
    B = 2
    feat = seeded_tensor(tag + ':feat', (B, cin, res, res), 1).requires_grad_()
    c0 = seeded_tensor(tag + ':c0', (B, 256), 1).requires_grad_()
    c1 = seeded_tensor(tag + ':c1', (B, 256), 1).requires_grad_()
    sm = torch.sigmoid(seeded_tensor(tag + ':m', (B, 1, res, res), 1)).requires_grad_()
    out, m = O.sagb_block(sd, '', feat, (c0, c1), sm, cin != cout, pm)
    assert_close_fp(tag + '/out', fp(out), g[tag + '/out'], RT, AT)
    loss = (out * seeded_tensor(tag + ':r', out.shape, 2)).sum()
    if pm:
        assert_close_fp(tag + '/mask', fp(m), g[tag + '/mask'], RT, AT)
        loss = loss + (m * seeded_tensor(tag + ':rm', m.shape, 2)).sum()
    loss.backward()
    for nm, t in [('feat', feat), ('c0', c0), ('c1', c1), ('m', sm)]:
        assert_close_fp(nm, fp(t.grad), g[tag + '/dinput/' + nm], RT, AT)
    _check_grads(tag, sd)
    for k, v in sd.items():
        if 'running' in k:
            assert_close_fp(k, fp(v), g[tag + '/after/' + k], RT, AT)


def test_cum_block():
    g = golden()
    sd = _req(golden_state('cum', 12))
    prev = seeded_tensor('cum:prev', (2, 16, 4, 4), 1).requires_grad_()
    cur = seeded_tensor('cum:cur', (2, 8, 8, 8), 1).requires_grad_()
    out = O.cum_block(sd, '', prev, cur)
    assert_close_fp('out', fp(out), g['cum/out'], RT, AT)
    (out * seeded_tensor('cum:r', out.shape, 2)).sum().backward()
    assert_close_fp('dprev', fp(prev.grad), g['cum/dinput/prev'], RT, AT)
    assert_close_fp('dcur', fp(cur.grad), g['cum/dinput/cur'], RT, AT)
    _check_grads('cum', sd)


@pytest.mark.parametrize('tag,fin,fout', [('resd_sc', 8, 16), ('resd_id', 16, 16)])
def test_resd(tag, fin, fout):
    g = golden()
    sd = _req(golden_state(tag, 13))
    x = seeded_tensor(tag + ':x', (2, fin, 8, 8), 1).requires_grad_()
    out = O.res_d(sd, '', x, fin, fout)
    assert_close_fp('out', fp(out), g[tag + '/out'], RT, AT)
    (out * seeded_tensor(tag + ':r', out.shape, 2)).sum().backward()
    assert_close_fp('dx', fp(x.grad), g[tag + '/dinput/x'], RT, AT)
    _check_grads(tag, sd)


def test_disc_heads():
    g = golden()
    sd = _req(golden_state('discsent', 14))
    f = seeded_tensor('ds:f', (2, 32, 4, 4), 1).requires_grad_()
    c = seeded_tensor('ds:c', (2, 256), 1).requires_grad_()
    out = O.disc_sent(sd, f, c, p='')
    assert_close_fp('ds', fp(out), g['discsent/out'], RT, AT)
    out.sum().backward()
    assert_close_fp('df', fp(f.grad), g['discsent/dinput/f'], RT, AT)
    assert_close_fp('dc', fp(c.grad), g['discsent/dinput/c'], RT, AT)
    _check_grads('discsent', sd)

    sd = _req(golden_state('disccond', 15))
    f = seeded_tensor('dc:f', (2, 32, 4, 4), 1).requires_grad_()
    c = seeded_tensor('dc:c', (2, 256), 1).requires_grad_()
    pair, cls = O.disc_cond(sd, f, c, p='')
    assert_close_fp('pair', fp(pair), g['disccond/pair'], RT, AT)
    assert_close_fp('cls', fp(cls), g['disccond/cls'], RT, AT)
    (pair.sum() + (cls * seeded_tensor('dc:r', cls.shape, 2)).sum()).backward()
    assert_close_fp('df', fp(f.grad), g['disccond/dinput/f'], RT, AT)
    assert_close_fp('dc', fp(c.grad), g['disccond/dinput/c'], RT, AT)
    _check_grads('disccond', sd)


def test_attr_enhance():
    g = golden()
    sd = _req(golden_state('attr', 16))
    s = seeded_tensor('ae:s', (2, 256), 1).requires_grad_()
    a = seeded_tensor('ae:a', (2, 3, 256), 1).requires_grad_()
    _, att = O.attr_enhance(sd, s, a)
    merged = O.attr_merge(att)
    assert_close_fp('att', fp(att), g['attr/att'], RT, AT)
    assert_close_fp('merged', fp(merged), g['attr/merged'], RT, AT)
    (merged * seeded_tensor('ae:r', merged.shape, 2)).sum().backward()
    assert_close_fp('ds', fp(s.grad), g['attr/dinput/s'], RT, AT)
    assert_close_fp('da', fp(a.grad), g['attr/dinput/a'], RT, AT)
    _check_grads('attr', sd)


def test_syncbn_single():
    g = golden()
    sd = _req(golden_state('syncbn', 17))
    x = seeded_tensor('bn:x', (4, 8, 5, 5), 1).requires_grad_()
    y = O.sync_bn(x, sd, '')
    assert_close_fp('y', fp(y), g['syncbn/out'], RT, AT)
    (y * seeded_tensor('bn:r', y.shape, 2)).sum().backward()
    assert_close_fp('dx', fp(x.grad), g['syncbn/dinput/x'], RT, AT)
    _check_grads('syncbn', sd)
    assert_close_fp('rm', fp(sd['running_mean']), g['syncbn/after/running_mean'], RT, AT)
    assert_close_fp('rv', fp(sd['running_var']), g['syncbn/after/running_var'], RT, AT)


def test_syncbn_multi_formula():
    """The cross-replica formula (batchnorm.py:113-125) differs from the
    single-device one only by clamp(var, eps) vs var+eps: for well-conditioned
    data they agree to ~eps/var."""
    sd1 = golden_state('syncbn', 17)
    sd2 = golden_state('syncbn', 17)
    x = seeded_tensor('bn:x', (4, 8, 5, 5), 1)
    y1 = O.sync_bn(x, sd1, '', mode='single')
    y2 = O.sync_bn(x, sd2, '', mode='multi')
    assert torch.allclose(y1, y2, rtol=1e-4, atol=1e-4)
    assert torch.allclose(sd1['running_var'], sd2['running_var'], rtol=1e-6, atol=1e-7)


def test_gen_forward_backward():
    g = golden()
    sd = _req(golden_state('gen', 21))
    z = seeded_tensor('g:z', (2, 100), 1)
    s = seeded_tensor('g:s', (2, 256), 1).requires_grad_()
    a = seeded_tensor('g:a', (2, 256), 1).requires_grad_()
    imgs = O.gen_forward(sd, z, s, a, 8)
    loss = 0
    for k, im in enumerate(imgs):
        assert_close_fp('img%d' % k, fp(im), g['gen/img%d' % k], 5e-4, 5e-5)
        loss = loss + (im * seeded_tensor('g:r%d' % k, im.shape, 2)).sum()
    loss.backward()
    assert_close_fp('ds', fp(s.grad), g['gen/dinput/s'], 1e-3, 1e-4)
    assert_close_fp('da', fp(a.grad), g['gen/dinput/a'], 1e-3, 1e-4)
    _check_grads('gen', sd, 2e-3, 2e-4)
    for k, v in sd.items():
        if 'running' in k:
            assert_close_fp(k, fp(v), g['gen/after/' + k], 1e-4, 1e-5)


@pytest.mark.parametrize('kind', [64, 128, 256])
def test_dis_and_gradient_penalty(kind):
    g = golden()
    tag = 'dis%d' % kind
    sd = _req(golden_state(tag, 30 + kind))
    x = seeded_tensor(tag + ':x', (2, 3, kind, kind), 1, 'uniform')
    s = seeded_tensor(tag + ':s', (2, 256), 1)
    feat = O.dis_forward(sd, x, kind, 8)
    assert_close_fp('feat', fp(feat), g[tag + '/feat'], RT, AT)
    head = O.disc_cond if kind == 256 else O.disc_sent
    o = head(sd, feat, s)
    if kind == 256:
        assert_close_fp('out', fp(o[0]), g[tag + '/out'], RT, AT)
        assert_close_fp('cls', fp(o[1]), g[tag + '/cls'], RT, AT)
    else:
        assert_close_fp('out', fp(o), g[tag + '/out'], RT, AT)
    xi = x.clone().requires_grad_()
    si = s.clone().requires_grad_()
    out = head(sd, O.dis_forward(sd, xi, kind, 8), si)
    if kind == 256:
        out = out[0]
    gx, gs = torch.autograd.grad(out, (xi, si), torch.ones_like(out), create_graph=True)
    gp = O.gradient_penalty(gx, gs)
    assert_close_fp('gp', fp(gp.reshape(1)), g[tag + '/gp'].reshape(1), 1e-3, 0)
    gp.backward()
    _check_grads(tag + '_gp', sd, 2e-3, 1e-6)


def test_damsm_losses():
    g = golden()
    Bd = 6
    reg = seeded_tensor('dm:reg', (Bd, 256, 17, 17), 1).requires_grad_()
    words = seeded_tensor('dm:words', (Bd, 256, 12), 1).requires_grad_()
    cap_lens = torch.tensor([12, 5, 9, 12, 3, 7])
    class_ids = torch.LongTensor([3, 7, 3, 1, 7, 3])
    labels = torch.arange(Bd)
    w0, w1, maps = O.words_loss(reg, words, labels, cap_lens, class_ids, Bd)
    assert_close_fp('w0', fp(w0.reshape(1)), g['damsm/w0'].reshape(1), RT, AT)
    assert_close_fp('w1', fp(w1.reshape(1)), g['damsm/w1'].reshape(1), RT, AT)
    assert_close_fp('map0', fp(maps[0]), g['damsm/att_map0'], RT, AT)
    (w0 + 0.7 * w1).backward()
    assert_close_fp('dreg', fp(reg.grad), g['damsm/dreg'], 1e-3, 1e-6)
    assert_close_fp('dwords', fp(words.grad), g['damsm/dwords'], 1e-3, 1e-6)
    code = seeded_tensor('dm:code', (Bd, 256), 1).requires_grad_()
    rnn = seeded_tensor('dm:rnn', (Bd, 256), 1).requires_grad_()
    s0, s1 = O.sent_loss(code, rnn, labels, class_ids, Bd)
    assert_close_fp('s0', fp(s0.reshape(1)), g['damsm/s0'].reshape(1), RT, AT)
    assert_close_fp('s1', fp(s1.reshape(1)), g['damsm/s1'].reshape(1), RT, AT)
    (s0 + 0.3 * s1).backward()
    assert_close_fp('dcode', fp(code.grad), g['damsm/dcode'], 1e-3, 1e-6)
    assert_close_fp('drnn', fp(rnn.grad), g['damsm/drnn'], 1e-3, 1e-6)
    s0n, s1n = O.sent_loss(code.detach(), rnn.detach(), labels, None, Bd)
    assert np.allclose(s0n.item(), g['damsm/s0_nocls'], rtol=RT)
    assert np.allclose(s1n.item(), g['damsm/s1_nocls'], rtol=RT)
    w0n, w1n, _ = O.words_loss(reg.detach(), words.detach(), labels, cap_lens, None, Bd)
    assert np.allclose(w0n.item(), g['damsm/w0_nocls'], rtol=RT)
    assert np.allclose(w1n.item(), g['damsm/w1_nocls'], rtol=RT)
    q = seeded_tensor('dm:q', (3, 256, 7), 1)
    ctx = seeded_tensor('dm:ctx', (3, 256, 17, 17), 1)
    wc, att = O.func_attention(q, ctx, 5.0)
    assert_close_fp('fa_wc', fp(wc), g['damsm/fa_wc'], RT, AT)
    assert_close_fp('fa_att', fp(att), g['damsm/fa_att'], RT, AT)
    cos = O.cosine_similarity(seeded_tensor('dm:x1', (9, 256), 1), seeded_tensor('dm:x2', (9, 256), 1))
    assert_close_fp('cos', fp(cos), g['damsm/cos'], RT, AT)
    inp = seeded_tensor('dm:gin', (2, 32, 6, 6), 1)
    key = seeded_tensor('dm:gkey', (2, 32, 9), 1)
    val = seeded_tensor('dm:gval', (2, 32, 9), 1)
    gmask = torch.zeros(2, 9, dtype=torch.bool)
    gmask[0, 7:] = True
    gmask[1, 4:] = True
    gwc, gatt = O.global_attention_general(inp, key, val, gmask)
    assert_close_fp('gag_wc', fp(gwc), g['damsm/gag_wc'], RT, AT)
    assert_close_fp('gag_att', fp(gatt), g['damsm/gag_att'], RT, AT)


def test_labels_bit_exact():
    g = golden()
    r, f, m = O.prepare_labels(5)
    assert np.array_equal(r.numpy(), g['labels/real'])
    assert np.array_equal(f.numpy(), g['labels/fake'])
    assert np.array_equal(m.numpy(), g['labels/match'])
    lab = O.prepare_class_labels(5, 200, g['labels/cls_ids'])
    assert np.array_equal(lab.numpy(), g['labels/class'])   # id 0 -> last column


def test_rnn_encoder():
    g = golden()
    sd = golden_state('rnn', 41)
    caps = torch.as_tensor(g['rnn/caps']).long().reshape(4, 10)
    lens = torch.as_tensor(g['rnn/lens']).long()
    w, s = O.rnn_encoder(sd, caps, lens)
    assert_close_fp('words', fp(w), g['rnn/words'], 1e-4, 1e-6)
    assert_close_fp('sent', fp(s), g['rnn/sent'], 1e-4, 1e-6)


# tag: (batch, GF = DF, class count, USE_CLASS, stages, seed base) -- tests/golden/make_golden.py STEP_CASES
STEP_CASES = {'step': (4, 8, 10, True, 3, 50), 'stepnc': (4, 8, 10, False, 3, 110),
              'step12': (2, 12, 10, True, 3, 80), 'step1': (4, 8, 10, True, 1, 90)}


@pytest.mark.parametrize('tag', sorted(STEP_CASES))
def test_full_step(tag):
    """One d_update + g_update (train.py:437-502) with the stand-in image
    encoder: every post-Adam parameter and every logged loss.  'step' is the
    CUB-like W=8 step, 'stepnc' config C4's no-class-head discriminator,
    'step12' a width whose channel counts are not multiples of 32, 'step1'
    config C1's stage-1 slice."""
    g = golden()
    from oracle.eegan_oracle import STANDIN_SPEC
    B, W, ncls, disc_class, stages, sb = STEP_CASES[tag]
    nd = 3 if stages == 3 else 1
    sd_g = golden_state(tag + '_g', sb)
    sd_a = golden_state(tag + '_a', sb + 1)
    sd_ds = [golden_state(tag + '_d%d' % i, sb + 2 + i) for i in range(nd)]
    nets = O.OracleNets(sd_g, sd_a, sd_ds, W, W, disc_class, ncls)
    og, ods = O.make_adams(nets)
    sd_enc = seeded_state(STANDIN_SPEC, sb + 10)
    batch = synthetic_batch(B, seed=7, class_num=ncls, sizes=(64, 128, 256))
    words = seeded_tensor(tag + ':words', (B, 256, 18), 1)
    sent = seeded_tensor(tag + ':sent', (B, 256), 1)
    attrs = seeded_tensor(tag + ':attrs', (B, 3, 256), 1)
    unpair = seeded_tensor(tag + ':unpair', (B, 256), 1)
    fakes, drec, grec = O.train_step(nets, og, ods, batch, (words, sent, attrs, unpair),
                                     lambda x: O.standin_image_encoder(sd_enc, x), 10.0, 0.05, stages=stages)
    assert len(fakes) == nd
    for k, f in enumerate(fakes):
        assert_close_fp('fake%d' % k, fp(f), g[tag + '/fake%d' % k], 5e-4, 5e-5)
    names = json.loads(g[tag + '/scalars/names'].tobytes().decode())
    vals = dict(zip(names, g[tag + '/scalars/values']))
    for i, (_, gp) in enumerate(drec):
        assert np.isclose(gp.item(), vals['errD_%d/d_loss_gp' % i], rtol=2e-3), i
    _, errs, damsm = grec
    for i, e in enumerate(errs):
        assert np.isclose(e.item(), vals['errG/G_%d_fake_sent' % i], rtol=1e-3, atol=1e-5)
    assert np.isclose(damsm[0].item(), vals['errG/w_loss'], rtol=1e-4)
    assert np.isclose(damsm[1].item(), vals['errG/s_loss'], rtol=1e-4)
    assert np.isclose(damsm[2].item(), vals['errG/a_loss'], rtol=1e-4)
    assert ('errD_2/real_class' in vals) == (disc_class and nd == 3)
    # post-Adam parameters: Adam's first step moves each weight by ~lr*sign(g),
    # so the post-step weights are compared at lr-scale tolerance
    for nm, sd in [('g', sd_g), ('a', sd_a)] + [('d%d' % i, d) for i, d in enumerate(sd_ds)]:
        for k, v in sd.items():
            assert_close_fp(nm + ':' + k, fp(v), g[tag + '/after_%s/%s' % (nm, k)], 1e-4, 2e-5)
