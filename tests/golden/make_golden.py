#!/usr/bin/env python
"""Generate the golden vectors under tests/golden/ by importing the REFERENCE
(qikizh/EE-GAN at /root/reference) on CPU in the build container.

Run (build container only -- the reference never travels to the GPU box):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Import recipe: the reference's hot-path modules
(models.py, miscc/DAMSM_losses.py, sync_batchnorm/, train.py statics,
DAMSM.RNN_ENCODER) are imported unmodified.  Only OFF-path imports that are
absent from this image get inert in-memory stand-ins: ``easydict`` (a plain
attribute dict), ``tensorboardX`` (logging), ``torchvision`` (image IO /
transforms / the CNN_ENCODER backbone, which is therefore not fixtured) and
``nltk`` (tokenising).  No reference source is copied; only inputs and
outputs are written, as .npz data.

Weights come from oracle/seeding.py (seeded per state_dict key) so tests can
regenerate them without the reference; tensors larger than 4096 elements are
stored as fingerprints (oracle.seeding.summary).
"""
import json
import os
import sys
import types

import numpy as np
import torch

REF = '/root/reference'
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from oracle.seeding import seeded_state, state_spec, seeded_tensor, seeded_ints, summary  # noqa

torch.set_num_threads(8)
torch.set_default_dtype(torch.float32)


def install_stubs():
    class EasyDict(dict):
        def __getattr__(self, k):
            try:
                return self[k]
            except KeyError:
                raise AttributeError(k)

        def __setattr__(self, k, v):
            self[k] = v

    m = types.ModuleType('easydict')
    m.EasyDict = EasyDict
    sys.modules['easydict'] = m
    tb = types.ModuleType('tensorboardX')
    tb.SummaryWriter = lambda *a, **k: types.SimpleNamespace(add_scalar=lambda *a, **k: None)
    sys.modules['tensorboardX'] = tb
    tv = types.ModuleType('torchvision')
    for sub in ['transforms', 'models', 'utils']:
        sm = types.ModuleType('torchvision.' + sub)
        setattr(tv, sub, sm)
        sys.modules['torchvision.' + sub] = sm
    sys.modules['torchvision'] = tv
    nl = types.ModuleType('nltk')
    nt = types.ModuleType('nltk.tokenize')
    nt.RegexpTokenizer = object
    nl.tokenize = nt
    sys.modules['nltk'] = nl
    sys.modules['nltk.tokenize'] = nt


def import_reference():
    install_stubs()
    sys.path.insert(0, REF)
    from miscc.config import cfg
    cfg.CUDA = False
    import models
    import train
    import DAMSM
    import miscc.DAMSM_losses as L
    import sync_batchnorm as SB
    torch.Tensor.cuda = lambda self, *a, **k: self  # train.py:391 hard-codes .cuda()
    return cfg, models, train, DAMSM, L, SB


OUT = {}


def put(name, t, full=False):
    if isinstance(t, torch.Tensor):
        OUT[name] = t.detach().double().numpy().copy() if full else summary(t)
    else:
        OUT[name] = np.asarray(t)


def put_spec(name, sd):
    OUT[name + '/spec'] = np.frombuffer(json.dumps(state_spec(sd)).encode(), dtype=np.uint8)


def load_seeded(mod, seed):
    sd = seeded_state(state_spec(mod.state_dict()), seed)
    mod.load_state_dict(sd)
    return sd


def grads_of(mod, prefix):
    for k, p in mod.named_parameters():
        if p.grad is not None:
            put(prefix + '/grad/' + k, p.grad)


def main():
    cfg, models, train, DAMSM, L, SB = import_reference()
    B = 2

    # ---------------- blocks -------------------------------------------
    # affine_ssa + ReLU chain inside a SAGB block with learnable shortcut
    for tag, cin, cout, pm, res in [('sagb_sc', 16, 8, True, 8), ('sagb_id', 16, 16, True, 4),
                                    ('sagb_nomask', 8, 8, False, 8)]:
        blk = models.SAGB_Block(cin, cout, pred_mask=pm)
        load_seeded(blk, 11)
        put_spec(tag, blk.state_dict())
        feat = seeded_tensor(tag + ':feat', (B, cin, res, res), 1).requires_grad_()
        c0 = seeded_tensor(tag + ':c0', (B, 256), 1).requires_grad_()
        c1 = seeded_tensor(tag + ':c1', (B, 256), 1).requires_grad_()
        sm = torch.sigmoid(seeded_tensor(tag + ':m', (B, 1, res, res), 1)).requires_grad_()
        out, m = blk(feat, [c0, c1], sm)
        put(tag + '/out', out)
        loss = (out * seeded_tensor(tag + ':r', out.shape, 2)).sum()
        if pm:
            put(tag + '/mask', m)
            loss = loss + (m * seeded_tensor(tag + ':rm', m.shape, 2)).sum()
        loss.backward()
        for nm, t in [('feat', feat), ('c0', c0), ('c1', c1), ('m', sm)]:
            put(tag + '/dinput/' + nm, t.grad)
        grads_of(blk, tag)
        for k, v in blk.state_dict().items():
            if 'running' in k:
                put(tag + '/after/' + k, v)

    cum = models.Cum_Block(16, 8)
    load_seeded(cum, 12)
    put_spec('cum', cum.state_dict())
    prev = seeded_tensor('cum:prev', (B, 16, 4, 4), 1).requires_grad_()
    cur = seeded_tensor('cum:cur', (B, 8, 8, 8), 1).requires_grad_()
    out = cum(prev, cur)
    put('cum/out', out)
    (out * seeded_tensor('cum:r', out.shape, 2)).sum().backward()
    put('cum/dinput/prev', prev.grad)
    put('cum/dinput/cur', cur.grad)
    grads_of(cum, 'cum')

    for tag, fin, fout in [('resd_sc', 8, 16), ('resd_id', 16, 16)]:
        rd = models.resD(fin, fout)
        load_seeded(rd, 13)
        put_spec(tag, rd.state_dict())
        x = seeded_tensor(tag + ':x', (B, fin, 8, 8), 1).requires_grad_()
        out = rd(x)
        put(tag + '/out', out)
        (out * seeded_tensor(tag + ':r', out.shape, 2)).sum().backward()
        put(tag + '/dinput/x', x.grad)
        grads_of(rd, tag)

    ds = models.DiscSent(32, 256)
    load_seeded(ds, 14)
    put_spec('discsent', ds.state_dict())
    f = seeded_tensor('ds:f', (B, 32, 4, 4), 1).requires_grad_()
    c = seeded_tensor('ds:c', (B, 256), 1).requires_grad_()
    out = ds(f, c)
    put('discsent/out', out, full=True)
    out.sum().backward()
    put('discsent/dinput/f', f.grad)
    put('discsent/dinput/c', c.grad)
    grads_of(ds, 'discsent')

    dcnd = models.DiscCond(32, 256, class_nums=10)
    load_seeded(dcnd, 15)
    put_spec('disccond', dcnd.state_dict())
    f = seeded_tensor('dc:f', (B, 32, 4, 4), 1).requires_grad_()
    c = seeded_tensor('dc:c', (B, 256), 1).requires_grad_()
    pair, cls = dcnd(f, c)
    put('disccond/pair', pair, full=True)
    put('disccond/cls', cls, full=True)
    (pair.sum() + (cls * seeded_tensor('dc:r', cls.shape, 2)).sum()).backward()
    put('disccond/dinput/f', f.grad)
    put('disccond/dinput/c', c.grad)
    grads_of(dcnd, 'disccond')

    ae = models.ATTR_Enhance()
    load_seeded(ae, 16)
    put_spec('attr', ae.state_dict())
    s = seeded_tensor('ae:s', (B, 256), 1).requires_grad_()
    a = seeded_tensor('ae:a', (B, 3, 256), 1).requires_grad_()
    sent_o, att = ae(s, a)
    merged = models.ATTR_Enhance.attr_merge(att)
    put('attr/att', att)
    put('attr/merged', merged)
    (merged * seeded_tensor('ae:r', merged.shape, 2)).sum().backward()
    put('attr/dinput/s', s.grad)
    put('attr/dinput/a', a.grad)
    grads_of(ae, 'attr')

    bn = SB.SynchronizedBatchNorm2d(8)
    load_seeded(bn, 17)
    put_spec('syncbn', bn.state_dict())
    x = seeded_tensor('bn:x', (4, 8, 5, 5), 1).requires_grad_()
    y = bn(x)
    put('syncbn/out', y)
    (y * seeded_tensor('bn:r', y.shape, 2)).sum().backward()
    put('syncbn/dinput/x', x.grad)
    grads_of(bn, 'syncbn')
    put('syncbn/after/running_mean', bn.running_mean, full=True)
    put('syncbn/after/running_var', bn.running_var, full=True)

    # ---------------- Generator (ngf=8) --------------------------------
    G = models.Gen(8, 100)
    load_seeded(G, 21)
    put_spec('gen', G.state_dict())
    z = seeded_tensor('g:z', (B, 100), 1)
    s = seeded_tensor('g:s', (B, 256), 1).requires_grad_()
    a = seeded_tensor('g:a', (B, 256), 1).requires_grad_()
    imgs = G(z, s, a)
    loss = 0
    for k, im in enumerate(imgs):
        put('gen/img%d' % k, im)
        loss = loss + (im * seeded_tensor('g:r%d' % k, im.shape, 2)).sum()
    loss.backward()
    put('gen/dinput/s', s.grad)
    put('gen/dinput/a', a.grad)
    grads_of(G, 'gen')
    for k, v in G.state_dict().items():
        if 'running' in k:
            put('gen/after/' + k, v)

    # ---------------- Discriminators (ndf=8) + gradient penalty --------
    for kind in [64, 128, 256]:
        if kind == 256:
            D = models.Dis256(8, True, 10)
        else:
            D = getattr(models, 'Dis%d' % kind)(8)
        load_seeded(D, 30 + kind)
        tag = 'dis%d' % kind
        put_spec(tag, D.state_dict())
        x = seeded_tensor(tag + ':x', (B, 3, kind, kind), 1, 'uniform')
        s = seeded_tensor(tag + ':s', (B, 256), 1)
        netD = torch.nn.DataParallel(D)
        feat = netD(x)
        put(tag + '/feat', feat)
        o = netD.module.COND_DNET(feat, s)
        if kind == 256:
            put(tag + '/out', o[0], full=True)
            put(tag + '/cls', o[1], full=True)
        else:
            put(tag + '/out', o, full=True)
        gp = train.Trainer.MA_gradient_penalty(x, s, netD, kind == 256)
        put(tag + '/gp', gp, full=True)
        D.zero_grad()
        gp.backward()
        grads_of(D, tag + '_gp')

    # ---------------- DAMSM losses ------------------------------------
    Bd = 6
    reg = seeded_tensor('dm:reg', (Bd, 256, 17, 17), 1).requires_grad_()
    words = seeded_tensor('dm:words', (Bd, 256, 12), 1).requires_grad_()
    cap_lens = torch.tensor([12, 5, 9, 12, 3, 7])
    class_ids = torch.LongTensor([3, 7, 3, 1, 7, 3])    # deliberate collisions
    labels = torch.arange(Bd)
    put('damsm/cap_lens', cap_lens)
    put('damsm/class_ids', class_ids)
    w0, w1, maps = L.words_loss(reg, words, labels, cap_lens, class_ids, Bd)
    put('damsm/w0', w0, full=True)
    put('damsm/w1', w1, full=True)
    put('damsm/att_map0', maps[0])
    (w0 + 0.7 * w1).backward()
    put('damsm/dreg', reg.grad)
    put('damsm/dwords', words.grad)
    code = seeded_tensor('dm:code', (Bd, 256), 1).requires_grad_()
    rnn = seeded_tensor('dm:rnn', (Bd, 256), 1).requires_grad_()
    s0, s1 = L.sent_loss(code, rnn, labels, class_ids, Bd)
    put('damsm/s0', s0, full=True)
    put('damsm/s1', s1, full=True)
    (s0 + 0.3 * s1).backward()
    put('damsm/dcode', code.grad)
    put('damsm/drnn', rnn.grad)
    # no class ids
    s0n, s1n = L.sent_loss(code.detach(), rnn.detach(), labels, None, Bd)
    put('damsm/s0_nocls', s0n, full=True)
    put('damsm/s1_nocls', s1n, full=True)
    w0n, w1n, _ = L.words_loss(reg.detach(), words.detach(), labels, cap_lens, None, Bd)
    put('damsm/w0_nocls', w0n, full=True)
    put('damsm/w1_nocls', w1n, full=True)
    q = seeded_tensor('dm:q', (3, 256, 7), 1)
    ctx = seeded_tensor('dm:ctx', (3, 256, 17, 17), 1)
    wc, att = L.func_attention(q, ctx, 5.0)
    put('damsm/fa_wc', wc)
    put('damsm/fa_att', att)
    put('damsm/cos', L.cosine_similarity(seeded_tensor('dm:x1', (9, 256), 1),
                                          seeded_tensor('dm:x2', (9, 256), 1)), full=True)
    gag = L.GlobalAttentionGeneral(32, 32)
    inp = seeded_tensor('dm:gin', (2, 32, 6, 6), 1)
    key = seeded_tensor('dm:gkey', (2, 32, 9), 1)
    val = seeded_tensor('dm:gval', (2, 32, 9), 1)
    gmask = torch.zeros(2, 9, dtype=torch.bool)
    gmask[0, 7:] = True
    gmask[1, 4:] = True
    gag.applyMask(gmask)
    gwc, gatt = gag(inp, key, val)
    put('damsm/gag_wc', gwc)
    put('damsm/gag_att', gatt)

    # ---------------- labels -----------------------------------------
    rl, fl, ml = train.prepare_labels(5, 'cpu')
    put('labels/real', rl, full=True)
    put('labels/fake', fl, full=True)
    put('labels/match', ml, full=True)
    cids = np.array([1, 200, 0, 57, 57])
    put('labels/cls_ids', cids)
    put('labels/class', train.prepare_class_labels(5, 200, cids, 'cpu'), full=True)

    # ---------------- RNN_ENCODER ------------------------------------
    enc = DAMSM.RNN_ENCODER(50, nhidden=256)
    load_seeded(enc, 41)
    enc.eval()
    put_spec('rnn', enc.state_dict())
    caps = seeded_ints('rnn:caps', (4, 10), 1, 49, 1)
    lens = torch.tensor([10, 4, 7, 1])
    caps = caps * (torch.arange(10)[None] < lens[:, None]).long()
    put('rnn/caps', caps)
    put('rnn/lens', lens)
    with torch.no_grad():
        we, se = enc(caps, lens, enc.init_hidden(4))
    put('rnn/words', we)
    put('rnn/sent', se, full=True)

    # ---------------- one full d_update + g_update (W=8, B=4) --------
    step_case(models, train, L, cfg, 'step')

    np.savez_compressed(os.path.join(HERE, 'golden.npz'), **OUT)
    print('wrote', len(OUT), 'arrays')


def main_steps():
    """Round-2 step fixtures (tests/golden/golden_steps.npz): config C4's
    no-class-head step, a non-multiple-of-32 width, and the C1 stage-1 slice."""
    cfg, models, train, DAMSM, L, SB = import_reference()
    for tag in ('stepnc', 'step12', 'step1'):
        step_case(models, train, L, cfg, tag)
    np.savez_compressed(os.path.join(HERE, 'golden_steps.npz'), **OUT)
    print('wrote', len(OUT), 'arrays')


def gen_stage1(G, z, sent, attrs):
    """The harness's stage-1 slice of config C1 (the
    reference has no stage-1 mode): Gen.forward (models.py:225-252) up to
    img_64, calling the reference's own submodules in the reference's order,
    without the 128/256 branches."""
    out = G.fc(z).view(z.size(0), 8 * G.ngf, 4, 4)
    stage_mask = G.init_mask(out)
    out, stage_mask = G.blocks[0](out, [sent, sent], torch.sigmoid(stage_mask))
    for ix, scale in enumerate([8, 16, 32]):
        out, stage_mask = G.SAGB_progress(out, [sent, sent], stage_mask, scale, SAGB_block=G.blocks[ix + 1])
    x_32 = out
    x_64, stage_mask = G.SAGB_progress(x_32, [sent, attrs], stage_mask, 64, SAGB_block=G.blocks[4])
    return [G.get_image_64(G.cum_64(x_32, x_64))]


# name: (batch, GF = DF, class count, USE_CLASS, stages, seed base).  Seed
# bases are chosen so that no discriminator output of the d_update hinge
# terms lies within 0.03 of its kink (relu(1 - real), relu(1 + fake/mismatch),
# train.py:342-376): there bf16 rounding can switch a sample's gradient on or
# off, which flips Adam's sign-normalised first step for many weights (seed
# base 70 had a fake logit at -0.997; 110 keeps every one >= 0.36 away).
STEP_CASES = {
    'step': (4, 8, 10, True, 3, 50),      # round-1 fixture (CUB-like, class head on)
    'stepnc': (4, 8, 10, False, 3, 110),   # config C4's shape of the step: Dis256 with the DiscSent head, no class loss
    'step12': (2, 12, 10, True, 3, 80),   # widths that are not multiples of 32 (C3's W=48 takes the same padded-K paths)
    'step1': (4, 8, 10, True, 1, 90),     # config C1: the stage-1 slice (img_64, Dis64 only, DAMSM on img_64)
}


def step_case(models, train, L, cfg, tag='step'):
    """train.py:186-206 for one iteration with seeded weights and seeded
    text embeddings; the CNN_ENCODER (torchvision) is replaced by the
    stand-in image encoder of oracle.eegan_oracle.standin_image_encoder."""
    from oracle.eegan_oracle import STANDIN_SPEC, standin_image_encoder
    from oracle.seeding import synthetic_batch
    B, W, ncls, disc_class, stages, sb = STEP_CASES[tag]
    torch.manual_seed(0)
    G = models.Gen(W, 100)
    A = models.ATTR_Enhance()
    Ds = [models.Dis64(W), models.Dis128(W), models.Dis256(W, disc_class, ncls)][:3 if stages == 3 else 1]
    for i, m in enumerate([G, A] + Ds):
        load_seeded(m, sb + i)
    put_spec(tag + '_g', G.state_dict())
    put_spec(tag + '_a', A.state_dict())
    for i, d in enumerate(Ds):
        put_spec(tag + '_d%d' % i, d.state_dict())
    sd_enc = seeded_state(STANDIN_SPEC, sb + 10)

    T = object.__new__(train.Trainer)
    T.device = 'cpu'
    T.disc_class = disc_class
    T.class_nums = ncls
    T.batch_size = B
    T.d_class_coe = T.g_class_coe = 10.0
    T.DAMSM_coe = 0.05
    T.iters_cnt = 0
    rec = {}
    T.writer = types.SimpleNamespace(add_scalar=lambda n, v, it: rec.__setitem__(n, float(v)))
    netG = torch.nn.DataParallel(G)
    attr = torch.nn.DataParallel(A)
    T.netsD = [torch.nn.DataParallel(d) for d in Ds]
    T.image_encoder = lambda x: standin_image_encoder(sd_enc, x)
    T.optimizerG, T.optimizerDs = train.Trainer.load_optimizers(netG, T.netsD, attr)

    batch = synthetic_batch(B, seed=7, class_num=ncls, sizes=(64, 128, 256))
    words = seeded_tensor(tag + ':words', (B, 256, 18), 1)
    sent = seeded_tensor(tag + ':sent', (B, 256), 1)
    attrs = seeded_tensor(tag + ':attrs', (B, 3, 256), 1)
    unpair = seeded_tensor(tag + ':unpair', (B, 256), 1)
    cls_ids = batch['cls_ids'].numpy()
    class_labels = train.prepare_class_labels(B, ncls, cls_ids, 'cpu') if disc_class else None
    _, _, match = train.prepare_labels(B, 'cpu')
    _, att = attr(sent, attrs)
    attn_attr = attr.module.attr_merge(att)
    fakes = netG(batch['noise'], sent, attn_attr) if stages == 3 else gen_stage1(G, batch['noise'], sent, attn_attr)
    for k, f in enumerate(fakes):
        put(tag + '/fake%d' % k, f)
    T.d_update(batch['imgs'][:len(Ds)], fakes, sent, unpair, class_labels, True)
    T.g_update(fakes, sent, words, attn_attr, cls_ids, B, match, batch['cap_lens'], class_labels, True)
    OUT[tag + '/scalars/names'] = np.frombuffer(json.dumps(sorted(rec)).encode(), dtype=np.uint8)
    OUT[tag + '/scalars/values'] = np.array([rec[k] for k in sorted(rec)])
    for nm, m in [('g', G), ('a', A)] + [('d%d' % i, d) for i, d in enumerate(Ds)]:
        for k, v in m.state_dict().items():
            put(tag + '/after_%s/%s' % (nm, k), v)


if __name__ == '__main__':
    if '--steps' in sys.argv:
        main_steps()
    else:
        main()
