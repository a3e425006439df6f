"""Model-level parity on the GPU: the drop-in modules (ee-gan_amd/models.py,
miscc/DAMSM_losses.py, sync_batchnorm, DAMSM.py) against the golden vectors
captured from the reference (tests/golden/golden.npz) and the CPU oracle.

Tolerance (bf16 activations/gradients, fp32 accumulation, fp32 parameters):
relative L2 error over the fingerprinted entries <= TOL_FWD for forward
outputs, <= TOL_BWD for gradients.  Same-class masks / labels are bit-exact."""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from _util import golden, golden_state, fp, spec  # noqa: E402
from oracle.seeding import seeded_tensor, seeded_state, synthetic_batch, summary  # noqa: E402

TOL_FWD = 3e-2
TOL_BWD = 6e-2
# Gradients through a whole network are evaluated at bf16-rounded activations
# (shifted ReLU masks / BN statistics), which the reference's fp32 path does
# not see.  Simulating exactly that rounding inside the fp32 oracle (CPU)
# gives: generator input grads 8-9% rel-L2, Inception-v3 input grads 29%; the
# kernels here measure 9% and 30%.  Deep-gradient tolerances reflect that.
TOL_DEEP = 0.15
# Deep per-parameter gradients (whole generator, discriminator under the
# gradient penalty) are gated against their OWN bf16 simulation: the fp32
# oracle with every conv input / output and its gradient rounded to bf16
# (oracle.eegan_oracle.SIM_BF16) lands at sim_p from the reference; each
# parameter p must stay within max(TOL_SIM_FLOOR, TOL_SIM_FACTOR * sim_p),
# and the median over parameters of (GPU error / simulated error) within
# TOL_SIM_MEDIAN.  Generator: median sim 8.8%; the GPU / sim ratio has median
# 1.09 and worst 2.85 (a BN bias: a sum, one rounding realisation each).
TOL_SIM_FACTOR = 4.0
TOL_SIM_FLOOR = 0.06
TOL_SIM_MEDIAN = 1.6
# Residual gains (gamma, models.py:101,138,275): d gamma = <d out, h> over every
# activation of the block, the TRUE value being 1e-4..2e-2 of the
# Cauchy-Schwarz scale ||d out|| ||h|| (heavy cancellation).  A relative error
# e of d out moves it by up to e ||d out|| ||h||, so the gate is
# |got - ref| <= TOL_GAIN * ||d out|| ||h||  with the scale from the oracle
# (oracle.eegan_oracle.PROBE): measured 4e-3 on the GPU, 1.5e-3 simulated.
TOL_GAIN = 1e-2
# attr_key.bias has an identically-zero true gradient (softmax shift
# invariance): its gradient must vanish against the key weight's.
ZERO_GRAD = ('attr/grad/attr_key.bias',)
_LOG = []


def _rel_fp(got_t, ref_fp):
    got = np.asarray(fp(got_t.float().cpu()), np.float64).reshape(-1)
    ref = np.asarray(ref_fp, np.float64).reshape(-1)
    assert got.shape == ref.shape
    if ref.size > 4096 or ref.size == 6 + 512:
        got, ref = got[6:], ref[6:]
    return float(np.linalg.norm(got - ref) / max(np.linalg.norm(ref), 1e-30))


def _check(name, got_t, ref_fp, tol):
    e = _rel_fp(got_t, ref_fp)
    _LOG.append((name, e))
    print('PARITY %-50s rel_l2=%.3e (tol %.0e)' % (name, e, tol))
    assert e <= tol, (name, e)
    return e


@pytest.fixture(scope='module', autouse=True)
def _dump_log():
    yield
    out = os.environ.get('EEGAN_PARITY_LOG')
    if out:
        with open(out, 'a') as f:
            for n, e in _LOG:
                f.write('%s %.4e\n' % (n, e))


def _load(mod, name, seed, dev):
    mod.load_state_dict(golden_state(name, seed))
    return mod.to(dev)


def _oracle_grads(run, sim):
    """Parameter gradients of an oracle forward/backward `run(O)` -> (grads
    by key, gain scales ||d out|| ||h|| by gamma key); sim=True rounds every
    conv input / output and gradient to bf16."""
    from oracle import eegan_oracle as O
    O.SIM_BF16, O.PROBE = sim, {}
    try:
        sd = run(O)
        grads = {k: v.grad for k, v in sd.items() if v.grad is not None}
        scales = {p + 'gamma': float(out.grad.norm() * h.norm()) for p, (h, out) in O.PROBE.items()
                  if out.grad is not None}
    finally:
        O.SIM_BF16, O.PROBE = False, None
    return grads, scales


def _gain_check(key, got_t, ref, scale):
    got = float(got_t.float().reshape(-1)[0])
    ref = float(np.asarray(ref).reshape(-1)[0])
    e = abs(got - ref) / scale
    _LOG.append((key + ' (|err| / ||dout|| ||h||)', e))
    print('PARITY %-50s |err|/(|dout||h|)=%.3e (tol %.0e; rel %.3e)' % (key, e, TOL_GAIN, abs(got - ref) / abs(ref)))
    assert e <= TOL_GAIN, (key, e)


def _grads(tag, mod, tol=TOL_BWD, skip=(), median_tol=None, sim=None, gains=None):
    """Every parameter gradient of `mod` against golden `tag/grad/*`.  sim:
    {key: bf16-simulated rel error} -> per-parameter gates (TOL_SIM_*);
    gains: {gamma key: Cauchy-Schwarz scale} -> the TOL_GAIN gate."""
    g = golden()
    n = 0
    errs = []
    for k, p in mod.named_parameters():
        key = tag + '/grad/' + k
        if key not in g or any(s in k for s in skip):
            continue
        if p.grad is None:
            # no gradient path: the gradient penalty's biases reach its value only
            # through piecewise-constant leaky-relu masks (functional._mask_src); the
            # reference's own autograd returns exact zeros for them
            ref = np.asarray(g[key], np.float64)
            _LOG.append((key + ' (no gradient path; golden max |g|)', float(np.abs(ref).max())))
            print('PARITY %-50s no gradient path, golden max|g| = %.1e' % (key, float(np.abs(ref).max())))
            assert float(np.abs(ref).max()) == 0.0, key
            continue
        if key in ZERO_GRAD:
            ref_w = mod.get_parameter(k.replace('.bias', '.weight')).grad
            z = float(p.grad.norm() / ref_w.norm())
            _LOG.append((key + ' (||g|| / ||g_weight||)', z))
            print('PARITY %-50s ||g||/||g_w||=%.3e (true value 0)' % (key, z))
            assert z < 1e-4, (key, z)
            continue
        if gains is not None and k in gains:
            _gain_check(key, p.grad, g[key], gains[k])
            continue
        t = tol if sim is None else max(TOL_SIM_FLOOR, TOL_SIM_FACTOR * sim[k])
        e = _check(key, p.grad, g[key], t)
        errs.append(e if sim is None else e / max(sim[k], 1e-12))
        n += 1
    assert n > 0
    if median_tol is not None:
        assert float(np.median(errs)) <= median_tol, (tag, float(np.median(errs)))
    if sim is not None:
        med = float(np.median(errs))
        _LOG.append((tag + ' (median GPU / bf16-simulated error)', med))
        print('PARITY %-50s median GPU/sim error ratio %.3f (tol %.1f)' % (tag, med, TOL_SIM_MEDIAN))
        assert med <= TOL_SIM_MEDIAN, (tag, med)


@pytest.mark.parametrize('tag,cin,cout,pm,res', [('sagb_sc', 16, 8, True, 8), ('sagb_id', 16, 16, True, 4),
                                                 ('sagb_nomask', 8, 8, False, 8)])
def test_sagb_block(gpu, tag, cin, cout, pm, res):
    import models
    g = golden()
    blk = _load(models.SAGB_Block(cin, cout, pred_mask=pm), tag, 11, gpu)
    B = 2
    feat = seeded_tensor(tag + ':feat', (B, cin, res, res), 1).to(gpu).requires_grad_()
    c0 = seeded_tensor(tag + ':c0', (B, 256), 1).to(gpu).requires_grad_()
    c1 = seeded_tensor(tag + ':c1', (B, 256), 1).to(gpu).requires_grad_()
    sm = torch.sigmoid(seeded_tensor(tag + ':m', (B, 1, res, res), 1)).to(gpu).requires_grad_()
    out, m = blk(feat, [c0, c1], sm)
    _check(tag + '/out', out, g[tag + '/out'], TOL_FWD)
    loss = (out.float() * seeded_tensor(tag + ':r', out.shape, 2).to(gpu)).sum()
    if pm:
        _check(tag + '/mask', m, g[tag + '/mask'], TOL_FWD)
        loss = loss + (m * seeded_tensor(tag + ':rm', m.shape, 2).to(gpu)).sum()
    loss.backward()
    for nm, t in [('feat', feat), ('c0', c0), ('c1', c1), ('m', sm)]:
        _check(tag + '/d' + nm, t.grad, g[tag + '/dinput/' + nm], TOL_BWD)

    def run(O):
        sd = golden_state(tag, 11)
        for k, v in sd.items():
            if v.is_floating_point() and 'running' not in k:
                v.requires_grad_(True)
        inp = [seeded_tensor(tag + ':feat', (B, cin, res, res), 1), seeded_tensor(tag + ':c0', (B, 256), 1),
               seeded_tensor(tag + ':c1', (B, 256), 1), torch.sigmoid(seeded_tensor(tag + ':m', (B, 1, res, res), 1))]
        o, mo = O.sagb_block(sd, '', inp[0], (inp[1], inp[2]), inp[3], cin != cout, pm)
        lo = (o * seeded_tensor(tag + ':r', o.shape, 2)).sum()
        if pm:
            lo = lo + (mo * seeded_tensor(tag + ':rm', mo.shape, 2)).sum()
        lo.backward()
        return sd

    _grads(tag, blk, gains=_oracle_grads(run, False)[1])
    for k, v in blk.state_dict().items():
        if 'running' in k:
            _check(tag + '/' + k, v, g[tag + '/after/' + k], 1e-2)


def test_cum_resd_heads_attr(gpu):
    import models
    g = golden()
    cum = _load(models.Cum_Block(16, 8), 'cum', 12, gpu)
    prev = seeded_tensor('cum:prev', (2, 16, 4, 4), 1).to(gpu).requires_grad_()
    cur = seeded_tensor('cum:cur', (2, 8, 8, 8), 1).to(gpu).requires_grad_()
    out = cum(prev, cur)
    _check('cum/out', out, g['cum/out'], TOL_FWD)
    (out.float() * seeded_tensor('cum:r', out.shape, 2).to(gpu)).sum().backward()
    _check('cum/dprev', prev.grad, g['cum/dinput/prev'], TOL_BWD)
    _check('cum/dcur', cur.grad, g['cum/dinput/cur'], TOL_BWD)
    _grads('cum', cum)
    for tag, fin, fout in [('resd_sc', 8, 16), ('resd_id', 16, 16)]:
        rd = _load(models.resD(fin, fout), tag, 13, gpu)
        x = seeded_tensor(tag + ':x', (2, fin, 8, 8), 1).to(gpu).requires_grad_()
        out = rd(x)
        _check(tag + '/out', out, g[tag + '/out'], TOL_FWD)
        (out.float() * seeded_tensor(tag + ':r', out.shape, 2).to(gpu)).sum().backward()
        _check(tag + '/dx', x.grad, g[tag + '/dinput/x'], TOL_BWD)
        _grads(tag, rd, skip=('conv_s',) if fin == fout else ())
    ds = _load(models.DiscSent(32, 256), 'discsent', 14, gpu)
    f = seeded_tensor('ds:f', (2, 32, 4, 4), 1).to(gpu).requires_grad_()
    c = seeded_tensor('ds:c', (2, 256), 1).to(gpu).requires_grad_()
    o = ds(f, c)
    _check('discsent/out', o, g['discsent/out'], TOL_FWD)
    o.sum().backward()
    _check('discsent/df', f.grad, g['discsent/dinput/f'], TOL_BWD)
    _check('discsent/dc', c.grad, g['discsent/dinput/c'], TOL_BWD)
    _grads('discsent', ds)
    dc = _load(models.DiscCond(32, 256, class_nums=10), 'disccond', 15, gpu)
    f = seeded_tensor('dc:f', (2, 32, 4, 4), 1).to(gpu).requires_grad_()
    c = seeded_tensor('dc:c', (2, 256), 1).to(gpu).requires_grad_()
    pair, cls = dc(f, c)
    _check('disccond/pair', pair, g['disccond/pair'], TOL_FWD)
    _check('disccond/cls', cls, g['disccond/cls'], TOL_FWD)
    (pair.sum() + (cls * seeded_tensor('dc:r', cls.shape, 2).to(gpu)).sum()).backward()
    _check('disccond/df', f.grad, g['disccond/dinput/f'], TOL_BWD)
    _check('disccond/dc', c.grad, g['disccond/dinput/c'], TOL_BWD)
    _grads('disccond', dc)
    ae = _load(models.ATTR_Enhance(), 'attr', 16, gpu)
    s = seeded_tensor('ae:s', (2, 256), 1).to(gpu).requires_grad_()
    a = seeded_tensor('ae:a', (2, 3, 256), 1).to(gpu).requires_grad_()
    _, att = ae(s, a)
    merged = models.ATTR_Enhance.attr_merge(att)
    _check('attr/att', att, g['attr/att'], 1e-4)
    _check('attr/merged', merged, g['attr/merged'], 1e-4)
    (merged * seeded_tensor('ae:r', merged.shape, 2).to(gpu)).sum().backward()
    _check('attr/ds', s.grad, g['attr/dinput/s'], 1e-4)
    _check('attr/da', a.grad, g['attr/dinput/a'], 1e-4)
    _grads('attr', ae, 1e-4)


def test_syncbn_module(gpu):
    from sync_batchnorm import SynchronizedBatchNorm2d
    g = golden()
    bn = _load(SynchronizedBatchNorm2d(8), 'syncbn', 17, gpu)
    x = seeded_tensor('bn:x', (4, 8, 5, 5), 1).to(gpu).requires_grad_()
    y = bn(x)
    _check('syncbn/out', y, g['syncbn/out'], TOL_FWD)
    (y.float() * seeded_tensor('bn:r', y.shape, 2).to(gpu)).sum().backward()
    _check('syncbn/dx', x.grad, g['syncbn/dinput/x'], TOL_BWD)
    _grads('syncbn', bn, 1e-2)
    _check('syncbn/rm', bn.running_mean, g['syncbn/after/running_mean'], 1e-2)
    _check('syncbn/rv', bn.running_var, g['syncbn/after/running_var'], 1e-2)
    assert x.grad.dtype == torch.float32 and x.grad.shape == x.shape


@pytest.mark.parametrize('affine', [True, False])
def test_syncbn_multi_device_formula(gpu, monkeypatch, affine):
    """The kernels' multi-device SyncBN numerics (bn_finalize clamp mode,
    selected at world 1 by Fn.SYNC_BN_FORCE_MULTI / EEGAN_SYNCBN_MULTI=1)
    against the oracle's restatement of sync_batchnorm/batchnorm.py:57-75,
    113-125: clamp(var_biased, eps)^-1/2, running_var from the unbiased
    variance, and the gradient flowing through the batch statistics (zero
    through the clamp).  Channel 3 is constant up to 1e-4 noise (variance
    below eps), so the clamp branch and its zero gradient are exercised.
    affine=False is affine_ssa's modulated path (mode 1, gamma = beta = 0)."""
    from sync_batchnorm import SynchronizedBatchNorm2d
    from eegan_hip import functional as Fn
    from oracle import eegan_oracle as O
    monkeypatch.setattr(Fn, 'SYNC_BN_FORCE_MULTI', True)
    C = 8
    x = seeded_tensor('bnm:x', (4, C, 5, 5), 1) * 0.7 + 0.3
    x[:, 3] = 0.5 + 1e-4 * seeded_tensor('bnm:c', (4, 5, 5), 1)
    x = x.to(torch.bfloat16).float()            # the kernels read bf16 activations
    r = seeded_tensor('bnm:r', (4, C, 5, 5), 2).to(torch.bfloat16).float()
    bn = SynchronizedBatchNorm2d(C, affine=affine)
    sd = {'running_mean': seeded_tensor('bnm:rm', (C,), 1) * 0.1, 'running_var': 1 + seeded_tensor('bnm:rv', (C,), 1).abs()}
    if affine:
        sd['weight'] = 1 + 0.2 * seeded_tensor('bnm:w', (C,), 1)
        sd['bias'] = 0.1 * seeded_tensor('bnm:b', (C,), 1)
    bn.load_state_dict(sd, strict=False)
    bn = bn.to(gpu)
    xd = x.to(gpu).requires_grad_()
    if affine:
        y = bn(xd)
    else:
        zeros = torch.zeros(4, C, device=gpu)
        y = bn.modulate(xd, zeros, zeros, torch.ones(4, 1, 5, 5, device=gpu))
    (y.float() * r.to(gpu)).sum().backward()
    sdo = {k: v.clone() for k, v in sd.items()}
    for k in ('weight', 'bias'):
        if k in sdo:
            sdo[k].requires_grad_(True)
    xo = x.clone().requires_grad_()
    yo = O.sync_bn(xo, sdo, '', affine=affine, mode='multi')
    (yo * r).sum().backward()
    assert torch.isfinite(y.float()).all() and torch.isfinite(xd.grad).all()
    _check('syncbn_multi/out', y, summary(yo.detach()), TOL_FWD)
    _check('syncbn_multi/dx', xd.grad, summary(xo.grad), TOL_BWD)
    # channel 3: inv_std = eps^-1/2 (clamped) and no gradient through the variance
    assert abs(float(y.float()[:, 3].abs().max()) - float(yo.detach()[:, 3].abs().max())) < 2e-2
    _check('syncbn_multi/rm', bn.running_mean, summary(sdo['running_mean']), 1e-5)
    _check('syncbn_multi/rv', bn.running_var, summary(sdo['running_var']), 1e-5)
    if affine:
        _check('syncbn_multi/dw', bn.weight.grad, summary(sdo['weight'].grad), 1e-2)
        _check('syncbn_multi/db', bn.bias.grad, summary(sdo['bias'].grad), 1e-2)


# Image max-abs gate (bf16 kernels with fp32 accumulation should
# stay within max |d| <= 2e-2, mean <= 5e-3 of the fp32 reference on images).  The
# HIP path holds activations AND conv weights in bf16; the survey measured
# all-bf16 (weights + activations) at max 4.2e-2 from fp64.  So the gate is the
# survey's 2e-2 or, where bf16 storage alone moves the images further, 1.2 x
# the fp32 oracle's own max |d| with every conv input / output and weight
# rounded to bf16 (oracle.SIM_BF16 + rounded weights) -- the bound is logged.
# Measured (profiles/r04_parity_log.txt): GPU / simulation = 2.59e-2 / 2.42e-2,
# 4.06e-2 / 3.89e-2, 3.51e-2 / 3.87e-2 (ratios 1.07, 1.04, 0.91).
TOL_IMG_SIM = 1.2
TOL_IMG_MAX, TOL_IMG_MEAN = 2e-2, 5e-3


def _image_maxabs_gate(imgs, z, s, a, W=8):
    import torch.nn.functional as F
    from oracle import eegan_oracle as O
    sd = golden_state('gen', 21)
    args = (z.cpu(), s.detach().cpu(), a.detach().cpu())
    with torch.no_grad():
        ref = O.gen_forward(sd, *args, W)
        orig = O.conv

        def conv_w(x, sd_, p, stride=1, pad=0, bias=False):
            w = sd_[p + 'weight'].to(torch.bfloat16).float()
            return O._r(F.conv2d(O._r(x), w, sd_.get(p + 'bias') if bias else None, stride, pad))
        O.SIM_BF16, O.conv = True, conv_w
        try:
            sim = O.gen_forward(sd, *args, W)
        finally:
            O.SIM_BF16, O.conv = False, orig
    for k, (im, r, sm) in enumerate(zip(imgs, ref, sim)):
        d = (im.float().cpu() - r).abs()
        ds = (sm - r).abs()
        bound = max(TOL_IMG_MAX, TOL_IMG_SIM * float(ds.max()))
        _LOG.append(('gen/img%d max|d|' % k, float(d.max())))
        _LOG.append(('gen/img%d mean|d|' % k, float(d.mean())))
        _LOG.append(('gen/img%d max|d| of the bf16 simulation' % k, float(ds.max())))
        print('PARITY gen/img%d max|d| %.3e (gate %.3e; bf16 simulation %.3e) mean|d| %.3e (gate %.0e)'
              % (k, float(d.max()), bound, float(ds.max()), float(d.mean()), TOL_IMG_MEAN))
        assert float(d.max()) <= bound, (k, float(d.max()), bound)
        assert float(d.mean()) <= TOL_IMG_MEAN, (k, float(d.mean()))


def test_generator(gpu):
    import models
    g = golden()
    G = _load(models.Gen(8, 100), 'gen', 21, gpu)
    z = seeded_tensor('g:z', (2, 100), 1).to(gpu)
    s = seeded_tensor('g:s', (2, 256), 1).to(gpu).requires_grad_()
    a = seeded_tensor('g:a', (2, 256), 1).to(gpu).requires_grad_()
    imgs = G(z, s, a)
    _image_maxabs_gate(imgs, z, s, a)
    loss = 0
    for k, im in enumerate(imgs):
        _check('gen/img%d' % k, im, g['gen/img%d' % k], TOL_FWD)
        loss = loss + (im.float() * seeded_tensor('g:r%d' % k, im.shape, 2).to(gpu)).sum()
    loss.backward()
    _check('gen/ds', s.grad, g['gen/dinput/s'], TOL_DEEP)
    _check('gen/da', a.grad, g['gen/dinput/a'], TOL_DEEP)
    def run(O):
        sd = golden_state('gen', 21)
        for k, v in sd.items():
            if v.is_floating_point() and 'running' not in k:
                v.requires_grad_(True)
        so, ao = seeded_tensor('g:s', (2, 256), 1), seeded_tensor('g:a', (2, 256), 1)
        ims = O.gen_forward(sd, seeded_tensor('g:z', (2, 100), 1), so, ao, 8)
        sum((im * seeded_tensor('g:r%d' % k, im.shape, 2)).sum() for k, im in enumerate(ims)).backward()
        return sd

    _, gains = _oracle_grads(run, False)
    sim_grads, _ = _oracle_grads(run, True)
    sim = {k: _rel_fp(v, g['gen/grad/' + k]) for k, v in sim_grads.items() if 'gen/grad/' + k in g}
    _grads('gen', G, sim=sim, gains=gains)
    for k, v in G.state_dict().items():
        if 'running' in k:
            _check('gen/' + k, v, g['gen/after/' + k], 2e-2)


def test_generator_branched_matches_single_stream(gpu):
    """Gen.forward_branched (stage 2-3 Cum_Block / image branches on a second
    stream, the trainer's GEN_SIDE) runs the same operations on the same inputs
    as the single-stream forward, created in the same order: images AND every
    gradient bit-identical (autograd orders the backward by node creation, so
    the multi-consumer sums -- x_64, x_128, the masks -- add in the same order
    whichever stream a node ran on)."""
    import models
    G = _load(models.Gen(8, 100), 'gen', 21, gpu)
    z = seeded_tensor('g:z', (2, 100), 1).to(gpu)
    side = torch.cuda.Stream()
    res = []
    for st in (None, side):
        G.side_stream = st
        G.zero_grad(set_to_none=True)
        s = seeded_tensor('g:s', (2, 256), 1).to(gpu).requires_grad_()
        a = seeded_tensor('g:a', (2, 256), 1).to(gpu).requires_grad_()
        imgs = G(z, s, a)
        loss = sum((im.float() * seeded_tensor('g:r%d' % k, im.shape, 2).to(gpu)).sum() for k, im in enumerate(imgs))
        loss.backward()
        torch.cuda.synchronize()
        res.append(([im.float().cpu() for im in imgs], s.grad.cpu(), a.grad.cpu(),
                    {n: p.grad.cpu().clone() for n, p in G.named_parameters() if p.grad is not None}))
    G.side_stream = None
    (i0, s0, a0, g0), (i1, s1, a1, g1) = res
    for x, y in zip(i0, i1):
        assert torch.equal(x, y)
    assert set(g0) == set(g1)
    assert torch.equal(s1, s0) and torch.equal(a1, a0)
    diff = [n for n in g0 if not torch.equal(g1[n], g0[n])]
    assert not diff, diff


def test_generator_grouped_mlps_match_per_layer(gpu, monkeypatch):
    """Fn.AffineMLPsFn (all affine_ssa MLPs in grouped launches) computes the
    same products in the same order as the per-layer LinearFn path: images
    and parameter gradients bit-identical; the conditioning gradients sum the
    per-MLP terms in another order (fp32 rounding only)."""
    import models
    from eegan_hip import functional as Fn
    G = _load(models.Gen(8, 100), 'gen', 21, gpu)
    z = seeded_tensor('g:z', (2, 100), 1).to(gpu)
    res = []
    for grouped in (False, True):
        monkeypatch.setattr(Fn, 'GROUPED_MLP', grouped)
        G.zero_grad(set_to_none=True)
        s = seeded_tensor('g:s', (2, 256), 1).to(gpu).requires_grad_()
        a = seeded_tensor('g:a', (2, 256), 1).to(gpu).requires_grad_()
        imgs = G(z, s, a)
        loss = sum((im.float() * seeded_tensor('g:r%d' % k, im.shape, 2).to(gpu)).sum() for k, im in enumerate(imgs))
        loss.backward()
        res.append(([im.float().cpu() for im in imgs], s.grad.cpu(), a.grad.cpu(),
                     {n: p.grad.cpu().clone() for n, p in G.named_parameters() if p.grad is not None}))
    (i0, s0, a0, g0), (i1, s1, a1, g1) = res
    for x, y in zip(i0, i1):
        assert torch.equal(x, y)
    assert set(g0) == set(g1)
    for n in g0:
        if 'fc_gamma' in n or 'fc_beta' in n:
            assert torch.equal(g0[n], g1[n]), n
        else:
            assert torch.allclose(g0[n], g1[n], rtol=1e-4, atol=1e-6), n
    assert torch.allclose(s0, s1, rtol=1e-4, atol=1e-6) and torch.allclose(a0, a1, rtol=1e-4, atol=1e-6)


def test_fused_activation_backward_matches_separate(gpu, monkeypatch):
    """Activation backward fused into the consuming conv's data gradient /
    ScaleAddFn (resD, D heads, Inception branch chains) against the separate
    act_bwd passes (EEGAN_FUSE_ACT_BWD=0).  The fused product is taken on the
    fp32 accumulator before the one bf16 rounding (the separate pass rounds
    twice), so values agree to bf16 rounding, not bit for bit."""
    import models
    from DAMSM import CNN_ENCODER
    from eegan_hip import functional as Fn
    from eegan_hip.tensor import to_nhwc_bf16
    from _util import rel_l2
    D = _load(models.Dis256(8, True, 10), 'dis256', 30 + 256, gpu)
    E = CNN_ENCODER(256).to(gpu)
    x = seeded_tensor('fa:x', (2, 3, 256, 256), 1, 'uniform').to(gpu)
    s = seeded_tensor('fa:s', (2, 256), 1).to(gpu)
    res = []
    for fuse in (False, True):
        monkeypatch.setattr(Fn, 'FUSE_ACT_BWD', fuse)
        D.zero_grad(set_to_none=True)
        xi = to_nhwc_bf16(x).detach().requires_grad_()
        pair, cls = D.COND_DNET(D(xi), s)
        (pair.sum() + cls.square().sum()).backward()
        xe = x.detach().clone().requires_grad_()
        feats, code = E(xe)
        (feats.square().sum() + code.sum()).backward()
        res.append((xi.grad.float().cpu(), xe.grad.cpu(),
                    {n: p.grad.cpu() for n, p in D.named_parameters() if p.grad is not None}))
    (gx0, ge0, gp0), (gx1, ge1, gp1) = res
    assert rel_l2(gx1, gx0) < 2e-2 and rel_l2(ge1, ge0) < 2e-2
    assert set(gp0) == set(gp1)
    for n in gp0:
        assert rel_l2(gp1[n], gp0[n]) < 2e-2, n


@pytest.mark.parametrize('knob', ['FUSE_GP_ADDS', 'FUSE_GP_ACT', 'FUSE_GP_GATE'])
def test_gradient_penalty_fused_adds_match_separate(gpu, monkeypatch, knob):
    """The gradient penalty's create_graph backward with resD's two input
    gradients summed in the conv epilogue (PoolConvBwdDataFn) and ScaleAdd's
    double backward in one pass (ScaleAddBwdFn) against the separate passes
    plus autograd adds (Fn.FUSE_GP_ADDS = False); and with the LeakyReLU
    backward folded into the consuming conv's data gradient
    (GatedConvBwdDataFn) against separate ActBwdFn passes
    (Fn.FUSE_GP_ACT = False); and with resD's last LeakyReLU folded into
    ScaleAdd's create_graph backward (ScaleAddGateBwdFn: gamma * g * act'(h)
    in one pass, its double backward in one more) against ScaleAddBwdFn plus
    conv_r[2]'s ActBwdFn (Fn.FUSE_GP_GATE = False): the same values, rounded
    to bf16 once instead of twice, so gradients agree to bf16 rounding."""
    import models
    from eegan_hip import functional as Fn
    from eegan_hip.trainer import Trainer
    from sync_batchnorm import DataParallelWithCallback
    from _util import rel_l2
    D = _load(models.Dis256(8, True, 10), 'dis256', 30 + 256, gpu)
    with torch.no_grad():
        for i, b in enumerate((D.block0, D.block1, D.block2, D.block3, D.block4, D.block5)):
            b.gamma.fill_(0.25 + 0.1 * i)    # non-zero gains: both ScaleAdd paths carry gradient
    netD = DataParallelWithCallback(D)
    x = seeded_tensor('gpf:x', (2, 3, 256, 256), 1, 'uniform').to(gpu)
    s = seeded_tensor('gpf:s', (2, 256), 1).to(gpu)
    res = []
    for fuse in (False, True):
        monkeypatch.setattr(Fn, knob, fuse)
        D.zero_grad(set_to_none=True)
        gp = Trainer.MA_gradient_penalty(Fn.ImageToNhwcFn.apply(x), s, netD, True)
        gp.backward()
        res.append((gp.detach().cpu(), {n: p.grad.cpu() for n, p in D.named_parameters() if p.grad is not None}))
    (v0, g0), (v1, g1) = res
    assert torch.allclose(v0, v1, rtol=2e-2)
    assert set(g0) == set(g1) and any('gamma' in n for n in g0)
    for n in g0:
        assert rel_l2(g1[n], g0[n]) < 3e-2, n


def test_gradient_penalty_second_backward_skips_forward_graph(gpu, monkeypatch):
    """Trainer.MA_gradient_penalty's first backward reads the leaky-relu masks'
    activations detached (functional._mask_src; GP_DETACH_MASKS): the second
    backward then runs no forward conv's backward -- before, autograd walked the
    whole forward graph with zero-filled gradients (a data and a weight
    gradient per conv, adding zeros).  The parameter gradients are the same
    bits (a gradient the walk no longer reaches is the exact zero it added:
    compared as zero), the data-gradient launches of the second backward drop
    to none."""
    import models
    from eegan_hip import functional as Fn
    from eegan_hip.trainer import Trainer
    from sync_batchnorm import DataParallelWithCallback
    D = _load(models.Dis256(8, True, 10), 'dis256', 30 + 256, gpu)
    netD = DataParallelWithCallback(D)
    x = seeded_tensor('gpd:x', (2, 3, 256, 256), 1, 'uniform').to(gpu)
    s = seeded_tensor('gpd:s', (2, 256), 1).to(gpu)
    calls = {'n': 0}
    orig = Fn.conv_bwd_data_raw

    def counted(*a, **k):
        calls['n'] += 1
        return orig(*a, **k)
    res = {}
    for on in (False, True):
        monkeypatch.setattr(Fn, 'GP_DETACH_MASKS', on)
        D.zero_grad(set_to_none=True)
        gp = Trainer.MA_gradient_penalty(Fn.ImageToNhwcFn.apply(x), s, netD, True)
        monkeypatch.setattr(Fn, 'conv_bwd_data_raw', counted)
        calls['n'] = 0
        gp.backward()
        torch.cuda.synchronize()
        monkeypatch.setattr(Fn, 'conv_bwd_data_raw', orig)
        res[on] = (calls['n'], {n: (p.grad.cpu() if p.grad is not None else torch.zeros_like(p).cpu())
                                for n, p in D.named_parameters()})
    assert res[True][0] == 0 < res[False][0], (res[True][0], res[False][0])
    for n, g_off in res[False][1].items():
        assert torch.equal(res[True][1][n], g_off), n


def test_inception_stacked_1x1_matches_separate(gpu, monkeypatch):
    """Inception blocks' shared-input 1x1 branches as one stacked conv
    (DAMSM._Stacked1x1) vs separate convs: identical forward (same K order per
    output channel), input gradient equal up to the summation order."""
    import DAMSM
    from _util import rel_l2
    E = DAMSM.CNN_ENCODER(256).to(gpu)
    x = seeded_tensor('s1:x', (2, 3, 128, 128), 1, 'uniform').to(gpu)
    res = []
    for fuse in (False, True):
        monkeypatch.setattr(DAMSM, 'FUSE_1X1', fuse)
        xe = x.detach().clone().requires_grad_()
        feats, code = E(xe)
        (feats.square().sum() + code.sum()).backward()
        res.append((feats.cpu(), code.cpu(), xe.grad.cpu()))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    assert rel_l2(res[1][2], res[0][2]) < 2e-2


@pytest.mark.parametrize('kind', [64, 128, 256])
def test_discriminator_and_gradient_penalty(gpu, kind):
    import models
    from eegan_hip import functional as Fn
    from sync_batchnorm import DataParallelWithCallback
    g = golden()
    tag = 'dis%d' % kind
    D = models.Dis256(8, True, 10) if kind == 256 else getattr(models, 'Dis%d' % kind)(8)
    D = _load(D, tag, 30 + kind, gpu)
    x = seeded_tensor(tag + ':x', (2, 3, kind, kind), 1, 'uniform').to(gpu)
    s = seeded_tensor(tag + ':s', (2, 256), 1).to(gpu)
    netD = DataParallelWithCallback(D)
    feat = netD(x)
    _check(tag + '/feat', feat, g[tag + '/feat'], TOL_FWD)
    o = netD.module.COND_DNET(feat, s)
    if kind == 256:
        _check(tag + '/out', o[0], g[tag + '/out'], TOL_FWD)
        _check(tag + '/cls', o[1], g[tag + '/cls'], TOL_FWD)
    else:
        _check(tag + '/out', o, g[tag + '/out'], TOL_FWD)
    from eegan_hip.trainer import Trainer
    gp = Trainer.MA_gradient_penalty(Fn.ImageToNhwcFn.apply(x), s, netD, kind == 256)
    _check(tag + '/gp', gp.reshape(1), g[tag + '/gp'].reshape(1), 0.05)
    D.zero_grad()
    gp.backward()
    _grads(tag + '_gp', D, TOL_DEEP)


@pytest.mark.parametrize('disc_class', [True, False])
def test_d_loss_real_early_matches_batched(gpu, disc_class):
    """trainer.DREAL_EARLY: d_loss split into its real-image share (one D pass
    over the real images, real + mismatch heads) and its fake-image share,
    back-propagated one after the other into the same FlatAdam gradient, gives
    the loss values and the parameter gradient of the batched d_loss
    (train.py:336-376) -- the same per-sample sums in another accumulation
    order.  Full-size Dis256 (DF=32, batch 16)."""
    import models
    from eegan_hip import functional as Fn
    from eegan_hip.trainer import Trainer
    from eegan_hip.optim import FlatAdam
    from sync_batchnorm import DataParallelWithCallback
    torch.manual_seed(5)
    B, ncls = 16, 200
    D = models.Dis256(32, disc_class, ncls).to(gpu)
    netD = DataParallelWithCallback(D)
    opt = FlatAdam([p for p in D.parameters() if p.requires_grad], lr=4e-4, betas=(0.0, 0.9))
    real = Fn.ImageToNhwcFn.apply(seeded_tensor('dre:x', (B, 3, 256, 256), 1, 'uniform').to(gpu))
    fake = Fn.ImageToNhwcFn.apply(seeded_tensor('dre:f', (B, 3, 256, 256), 2, 'uniform').to(gpu))
    sent = seeded_tensor('dre:s', (B, 256), 1).to(gpu)
    wrong = seeded_tensor('dre:w', (B, 256), 2).to(gpu)
    labels = torch.zeros(B, ncls, device=gpu)
    labels[torch.arange(B), torch.arange(B) * 7 % ncls] = 1
    opt.zero_grad()
    if disc_class:
        v = Trainer.d_loss_class(real, fake, sent, wrong, labels, netD)
        loss = v[0] + (v[1] + v[2]) / 2.0 + (v[3] + v[4] + v[5]) / 3.0 * 10.0
        ref_vals = [v[0], v[2], v[1], v[3], v[5], v[4]]   # real, mismatch, fake per kind
    else:
        v = Trainer.d_loss(real, fake, sent, wrong, netD)
        loss = v[0] + (v[1] + v[2]) / 2.0
        ref_vals = [v[0], v[2], v[1]]
    loss.backward(inputs=opt.params)
    g_ref = opt.gflat.clone()
    opt.zero_grad()
    r = Trainer.d_loss_real(real, sent, wrong, labels, netD, disc_class)
    part = r[0] + r[1] / 2.0 + ((r[2] + r[3]) / 3.0 * 10.0 if disc_class else 0.0)
    part.backward(inputs=opt.params)
    f = Trainer.d_loss_fake(fake, sent, labels, netD, disc_class)
    (f[0] / 2.0 + (f[1] / 3.0 * 10.0 if disc_class else 0.0)).backward(inputs=opt.params)
    torch.cuda.synchronize()
    vals = [r[0], r[1], f[0]] + ([r[2], r[3], f[1]] if disc_class else [])
    for a, b in zip(vals, ref_vals):
        a, b = float(a.detach()), float(b.detach())
        assert abs(a - b) <= 1e-3 * max(1.0, abs(b)), (a, b)
    a, b = opt.gflat.cpu().double(), g_ref.cpu().double()
    err = float((a - b).norm() / b.norm())
    print('d_loss real-early vs batched: gradient rel-L2 %.2e' % err)
    assert err < 5e-3


# DAMSM words similarity on bf16 MFMA (csrc/damsm.hip): the attention logits
# S = ctx q^T use split-bf16 products (hi*hi + lo*hi + hi*lo, ~fp32), the
# context C = A2 ctx and the backward contractions plain bf16 with fp32
# accumulation.  Emulating exactly that rounding in fp32 torch on these golden
# inputs gives losses within 7e-5 relative and d regions / d words within
# 3.6e-3 rel-L2 of the fp32 reference (1.0e-4 / 2.5e-3 at realistic region
# scales); the gates below leave ~3x headroom.
TOL_DAMSM_LOSS = 3e-4
TOL_DAMSM_GRAD = 1.2e-2


def test_damsm_losses(gpu):
    from miscc.DAMSM_losses import words_loss, sent_loss
    g = golden()
    Bd = 6
    reg = seeded_tensor('dm:reg', (Bd, 256, 17, 17), 1).to(gpu).requires_grad_()
    words = seeded_tensor('dm:words', (Bd, 256, 12), 1).to(gpu).requires_grad_()
    cap_lens = torch.tensor([12, 5, 9, 12, 3, 7]).to(gpu)
    class_ids = torch.LongTensor([3, 7, 3, 1, 7, 3])
    labels = torch.arange(Bd).to(gpu)
    w0, w1, maps = words_loss(reg, words, labels, cap_lens, class_ids, Bd)
    _check('damsm/w0', w0.reshape(1), g['damsm/w0'].reshape(1), TOL_DAMSM_LOSS)
    _check('damsm/w1', w1.reshape(1), g['damsm/w1'].reshape(1), TOL_DAMSM_LOSS)
    _check('damsm/att_map0', maps[0], g['damsm/att_map0'], 2e-3)
    (w0 + 0.7 * w1).backward()
    _check('damsm/dreg', reg.grad, g['damsm/dreg'], TOL_DAMSM_GRAD)
    _check('damsm/dwords', words.grad, g['damsm/dwords'], TOL_DAMSM_GRAD)
    code = seeded_tensor('dm:code', (Bd, 256), 1).to(gpu).requires_grad_()
    rnn = seeded_tensor('dm:rnn', (Bd, 256), 1).to(gpu).requires_grad_()
    s0, s1 = sent_loss(code, rnn, labels, class_ids, Bd)
    _check('damsm/s0', s0.reshape(1), g['damsm/s0'].reshape(1), 1e-5)
    _check('damsm/s1', s1.reshape(1), g['damsm/s1'].reshape(1), 1e-5)
    (s0 + 0.3 * s1).backward()
    _check('damsm/dcode', code.grad, g['damsm/dcode'], 1e-4)
    _check('damsm/drnn', rnn.grad, g['damsm/drnn'], 1e-4)
    s0n, s1n = sent_loss(code.detach(), rnn.detach(), labels, None, Bd)
    _check('damsm/s0_nocls', s0n.reshape(1), g['damsm/s0_nocls'].reshape(1), 1e-5)
    _check('damsm/s1_nocls', s1n.reshape(1), g['damsm/s1_nocls'].reshape(1), 1e-5)
    w0n, w1n, _ = words_loss(reg.detach(), words.detach(), labels, cap_lens, None, Bd)
    _check('damsm/w0_nocls', w0n.reshape(1), g['damsm/w0_nocls'].reshape(1), TOL_DAMSM_LOSS)
    _check('damsm/w1_nocls', w1n.reshape(1), g['damsm/w1_nocls'].reshape(1), TOL_DAMSM_LOSS)


@pytest.mark.parametrize('n_img,n_txt,T,off', [(3, 7, 20, 2), (16, 16, 18, 0), (2, 5, 32, 3),
                                               (32, 256, 18, 5)])   # C5's rank: 32 local x 256 global
def test_words_block_rectangular(gpu, n_img, n_txt, T, off):
    """The B_local x B_global block a data-parallel rank computes: rows for
    n_img images against n_txt captions (lengths 1..T, > 16 words use both
    word tiles), against the oracle's func_attention / cosine restatement at
    realistic region scale; attention maps of the pairs (j, j + off); the
    backward is deterministic (two runs bit-identical: no atomics)."""
    from eegan_hip import functional as Fn
    from oracle import eegan_oracle as O
    torch.manual_seed(n_img * 100 + n_txt)
    reg = torch.randn(n_img, 256, 17, 17) * 0.3
    words = torch.randn(n_txt, 256, T).tanh()
    lens = torch.randint(1, T + 1, (n_txt,))
    lens[0] = T
    lens[-1] = 1
    dsim = torch.randn(n_img, n_txt)
    # oracle: rows j (images) x columns i (captions)
    rr = reg.clone().requires_grad_()
    wr = words.clone().requires_grad_()
    cols, maps = [], {}
    for i in range(n_txt):
        w = int(lens[i])
        q = wr[i:i + 1, :, :w].expand(n_img, -1, -1)
        wc, att = O.func_attention(q, rr, O.GAMMA1)
        cos = O.cosine_similarity(q.transpose(1, 2).reshape(n_img * w, -1), wc.transpose(1, 2).reshape(n_img * w, -1))
        cols.append(torch.log(torch.exp(cos.reshape(n_img, w) * O.GAMMA2).sum(1, keepdim=True)))
        if 0 <= i - off < n_img:
            maps[i - off] = att[i - off]
    simr = torch.cat(cols, 1) * O.GAMMA3
    (simr * dsim).sum().backward()
    outs = []
    for _ in range(2):
        rd = reg.to(gpu).requires_grad_()
        wd = words.to(gpu).requires_grad_()
        sim, att = Fn.WordsSimFn.apply(rd, wd, lens.to(gpu), True, off)
        (sim * dsim.to(gpu)).sum().backward()
        outs.append((sim.detach().cpu(), att.cpu(), rd.grad.cpu(), wd.grad.cpu()))
    sim, att, dreg, dwords = outs[0]
    from _util import rel_l2
    assert (sim - simr.detach()).abs().max() < 2e-3 * simr.detach().abs().max()
    for j, m in maps.items():
        w = int(lens[j + off])
        assert rel_l2(att[j, :w].reshape(1, w, 17, 17), m.detach().reshape(1, w, 17, 17)) < 2e-3
    assert rel_l2(dreg, rr.grad) < TOL_DAMSM_GRAD, rel_l2(dreg, rr.grad)
    assert rel_l2(dwords, wr.grad) < TOL_DAMSM_GRAD, rel_l2(dwords, wr.grad)
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)


def test_rnn_encoder(gpu):
    import DAMSM
    g = golden()
    enc = _load(DAMSM.RNN_ENCODER(50, nhidden=256), 'rnn', 41, gpu).eval()
    caps = torch.as_tensor(g['rnn/caps']).long().reshape(4, 10).to(gpu)
    lens = torch.as_tensor(g['rnn/lens']).long().to(gpu)
    w, s = enc(caps, lens, enc.init_hidden(4))
    _check('rnn/words', w, g['rnn/words'], 1e-5)
    _check('rnn/sent', s, g['rnn/sent'], 1e-5)
    # the Trainer encodes captions + unpaired captions (and the attribute
    # phrases) as one batch: per-caption results must not depend on batching
    T = int(lens.max())
    w2, s2 = enc(torch.cat([caps, caps.flip(0)]), torch.cat([lens, lens.flip(0)]), None, max_len=T)
    assert torch.equal(w2[:4], w) and torch.equal(s2[:4], s)
    assert torch.equal(s2[4:], s.flip(0))


def test_cnn_encoder_vs_oracle(gpu):
    """Inception-v3 CNN_ENCODER vs the oracle restatement (parity unpinned by
    the reference: torchvision absent)."""
    import DAMSM
    from oracle import eegan_oracle as O
    torch.manual_seed(0)
    enc = DAMSM.CNN_ENCODER(256)
    sd = seeded_state([(k, tuple(v.shape)) for k, v in enc.state_dict().items()], 71)
    enc.load_state_dict(sd)
    enc = enc.to(gpu).eval()
    x = seeded_tensor('cnn:x', (2, 3, 64, 64), 1, 'uniform')
    xd = x.to(gpu).requires_grad_()
    feats, code = enc(xd)
    xr = x.clone().requires_grad_()
    fr, cr = O.cnn_encoder(sd, xr)
    e1 = _rel_fp(feats, summary(fr))
    e2 = _rel_fp(code, summary(cr))
    print('PARITY cnn/feats %.3e cnn/code %.3e' % (e1, e2))
    assert e1 < 5e-2 and e2 < 5e-2
    r1 = seeded_tensor('cnn:r1', fr.shape, 2)
    r2 = seeded_tensor('cnn:r2', cr.shape, 2)
    ((feats.float() * r1.to(gpu)).sum() + (code * r2.to(gpu)).sum()).backward()
    ((fr * r1).sum() + (cr * r2).sum()).backward()
    e3 = _rel_fp(xd.grad, summary(xr.grad))
    print('PARITY cnn/dx %.3e' % e3)
    assert e3 < 0.4   # bf16-activation simulation of the fp32 oracle: 0.29 (see TOL_DEEP note)


def test_cnn_encoder_stages(gpu):
    """Each Inception stage on the same bf16-rounded input vs the oracle."""
    import DAMSM
    from oracle import eegan_oracle as O
    from eegan_hip import functional as Fn
    enc = DAMSM.CNN_ENCODER(256)
    sd = seeded_state([(k, tuple(v.shape)) for k, v in enc.state_dict().items()], 71)
    enc.load_state_dict(sd)
    enc = enc.to(gpu).eval()
    stages = [
        ('Conv2d_1a_3x3', 3, 21, lambda t: O._basic_conv(sd, 'Conv2d_1a_3x3.', t, stride=2)),
        ('Conv2d_2b_3x3', 32, 9, lambda t: O._basic_conv(sd, 'Conv2d_2b_3x3.', t, pad=1)),
        ('Mixed_5b', 192, 9, lambda t: O._incA(sd, 'Mixed_5b.', t)),
        ('Mixed_6a', 288, 9, lambda t: O._incB(sd, 'Mixed_6a.', t)),
        ('Mixed_6b', 768, 7, lambda t: O._incC(sd, 'Mixed_6b.', t)),
        ('Mixed_7a', 768, 9, lambda t: O._incD(sd, 'Mixed_7a.', t)),
        ('Mixed_7b', 1280, 5, lambda t: O._incE(sd, 'Mixed_7b.', t)),
    ]
    bad = []
    for name, C, S, ref in stages:
        x = (torch.rand(2, C, S, S) * 2).to(torch.bfloat16).float()
        y = getattr(enc, name)(Fn.ImageToNhwcFn.apply(x.to(gpu)))
        yr = ref(x)
        e = _rel_fp(y, summary(yr))
        print('PARITY cnn-stage %-15s rel_l2=%.3e' % (name, e))
        if e > 2e-2:
            bad.append((name, e))
    x = (torch.rand(2, 3, 32, 32) * 2 - 1).to(torch.bfloat16).float()
    y = Fn.BilinearFn.apply(Fn.ImageToNhwcFn.apply(x.to(gpu)), 299, 299)
    yr = torch.nn.functional.interpolate(x, size=(299, 299), mode='bilinear', align_corners=False)
    e = _rel_fp(y, summary(yr))
    print('PARITY cnn-stage bilinear299 rel_l2=%.3e' % e)
    if e > 2e-2:
        bad.append(('bilinear', e))
    assert not bad, bad


# Full-step loss gates.  Losses evaluated before any parameter moved (the D
# hinge / class terms, the DAMSM losses) within TOL_STEP_LOSS (measured
# <= 1.4%).  The gradient penalty (after D's first Adam step) and the G hinge
# terms errG/G_i (after D's two steps) read a discriminator that Adam's first
# steps moved by ~lr * sign(grad) per weight WHATEVER the gradient's size, so
# the ~2% of weights whose gradient is within bf16 noise of zero can step the
# other way, and that step is a large part of those quantities (the update
# moves the penalty by 4-73% on these fixtures).  They are gated in units of
# the update's own effect U = ref - (the quantity at D's initial weights,
# fp32 oracle): |got - ref| <= TOL_STEP_LOSS |ref| + TOL_STEP_UPDATE |U|.
# Measured on the GPU up to 0.438 |U| (step/errD_2/d_loss_gp,
# profiles/r04_parity_log.txt; the other post-update terms <= 0.03 |U|); the
# fp32 oracle with bf16 activations AND bf16 conv weights lands at 0.30-0.39 |U|
# on the same term (tools/gp_sim_parity.py), so the gate
# keeps a 0.06 |U| margin over the measurement.
TOL_STEP_LOSS = 3e-2
TOL_STEP_UPDATE = 0.5
# Adam's first steps move each weight by ~lr * sign(grad), so post-step
# weights are compared by the direction of the move where the reference moved
# by > lr/2: measured sign agreement 0.980, gated at TOL_STEP_SIGN.
TOL_STEP_SIGN = 0.95


def _pre_update_values(tag, B, W, ncls, disc_class, stages, sb):
    """fp32 oracle values of the post-update losses at D's INITIAL weights:
    {'errG/G_i_fake_sent': ..., 'errD_i/d_loss_gp': ...}."""
    from oracle import eegan_oracle as O
    nd = 3 if stages == 3 else 1
    sd_g, sd_a = golden_state(tag + '_g', sb), golden_state(tag + '_a', sb + 1)
    sd_ds = [golden_state(tag + '_d%d' % i, sb + 2 + i) for i in range(nd)]
    nets = O.OracleNets(sd_g, sd_a, sd_ds, W, W, disc_class, ncls)
    batch = synthetic_batch(B, seed=7, class_num=ncls, sizes=(64, 128, 256))
    sent = seeded_tensor(tag + ':sent', (B, 256), 1)
    attrs = seeded_tensor(tag + ':attrs', (B, 3, 256), 1)
    _, att = O.attr_enhance(sd_a, sent, attrs)
    fakes = O.gen_forward(sd_g, batch['noise'], sent, O.attr_merge(att), W, 'single', stages)
    out = {}
    for i in range(nd):
        with torch.no_grad():
            o = nets.d_cond(i, nets.d_feat(i, fakes[i]), sent)
        out['errG/G_%d_fake_sent' % i] = -float((o[0] if (disc_class and i == 2) else o).mean())
        xi, si = batch['imgs'][i].clone().requires_grad_(), sent.clone().requires_grad_()
        o = nets.d_cond(i, nets.d_feat(i, xi), si)
        o = o[0] if (disc_class and i == 2) else o
        gx, gs = torch.autograd.grad(o, (xi, si), torch.ones_like(o))
        out['errD_%d/d_loss_gp' % i] = float(O.gradient_penalty(gx, gs))
    return out


# tag: (batch, GF = DF, class count, USE_CLASS, stages, seed base) -- tests/golden/make_golden.py STEP_CASES
STEP_CASES = {'step': (4, 8, 10, True, 3, 50), 'stepnc': (4, 8, 10, False, 3, 110),
              'step12': (2, 12, 10, True, 3, 80), 'step1': (4, 8, 10, True, 1, 90)}


def _standin_encoder(sd_enc, gpu):
    from eegan_hip import functional as Fn
    from eegan_hip.nn import Conv2d, Linear
    rconv = Conv2d(3, 256, 15, 15, 0, bias=False).to(gpu)
    rconv.weight.data.copy_(sd_enc['standin.regions.weight'].to(gpu))
    rconv.weight.requires_grad_(False)
    clin = Linear(256, 256).to(gpu)
    clin.weight.data.copy_(sd_enc['standin.code.weight'].to(gpu))
    clin.bias.data.copy_(sd_enc['standin.code.bias'].to(gpu))
    for p in clin.parameters():
        p.requires_grad_(False)

    def standin(x):
        if x.shape[-1] != 256:   # the stage-1 slice's img_64 (oracle.standin_image_encoder)
            x = Fn.BilinearFn.apply(x, 256, 256)
        r = rconv(x, out_f32=True)
        return r, clin(Fn.GlobalAvgPoolFn.apply(Fn.CastF32Bf16Fn.apply(r)))
    return standin


@pytest.mark.parametrize('tag', sorted(STEP_CASES))
def test_full_step(gpu, tag):
    """train.py:186-206 on the GPU vs the golden d_update + g_update captured
    from the reference (stand-in image encoder): losses and every post-Adam
    parameter.  'step': CUB-like W=8 step; 'stepnc': config C4's discriminator
    (Dis256 with the DiscSent head, USE_CLASS=False); 'step12': W=12, whose
    channel counts (12..192) are not multiples of 32 -- the padded-K paths
    config C3's W=48 takes; 'step1': config C1's stage-1 slice (Gen.stages=1,
    Dis64 only, DAMSM on img_64)."""
    import models
    from eegan_hip.trainer import Trainer
    from eegan_hip import functional as Fn
    from sync_batchnorm import DataParallelWithCallback
    from oracle.eegan_oracle import STANDIN_SPEC
    g = golden()
    B, W, ncls, disc_class, stages, sb = STEP_CASES[tag]
    nd = 3 if stages == 3 else 1
    G = _load(models.Gen(W, 100), tag + '_g', sb, gpu)
    G.stages = stages
    A = _load(models.ATTR_Enhance(), tag + '_a', sb + 1, gpu)
    makers = [lambda: models.Dis64(W), lambda: models.Dis128(W), lambda: models.Dis256(W, disc_class, ncls)]
    Ds = [_load(makers[i](), tag + '_d%d' % i, sb + 2 + i, gpu) for i in range(nd)]
    standin = _standin_encoder(seeded_state(STANDIN_SPEC, sb + 10), gpu)
    T = Trainer(DataParallelWithCallback(G), DataParallelWithCallback(A), [DataParallelWithCallback(d) for d in Ds],
                standin, None, B, disc_class=disc_class, class_nums=ncls, class_coe=10.0, sim_coe=0.05, device=gpu)
    batch = synthetic_batch(B, seed=7, class_num=ncls, sizes=(64, 128, 256))
    dbatch = {'imgs': [Fn.ImageToNhwcFn.apply(t.to(gpu)) for t in batch['imgs'][:nd]],
              'cls_ids': batch['cls_ids'].to(gpu), 'cap_lens': batch['cap_lens'].to(gpu)}
    words = seeded_tensor(tag + ':words', (B, 256, 18), 1).to(gpu)
    sent = seeded_tensor(tag + ':sent', (B, 256), 1).to(gpu)
    attrs = seeded_tensor(tag + ':attrs', (B, 3, 256), 1).to(gpu)
    unpair = seeded_tensor(tag + ':unpair', (B, 256), 1).to(gpu)
    fakes, _ = T.train_step(dbatch, noise=batch['noise'].to(gpu), emb=(words, sent, attrs, unpair), iter_rec=True)
    assert len(fakes) == nd
    for k, f in enumerate(fakes):
        _check('%s/fake%d' % (tag, k), f, g['%s/fake%d' % (tag, k)], TOL_FWD)
    names = json.loads(g[tag + '/scalars/names'].tobytes().decode())
    vals = dict(zip(names, g[tag + '/scalars/values']))
    assert set(T.records) == set(vals), (sorted(T.records), sorted(vals))
    pre = _pre_update_values(tag, B, W, ncls, disc_class, stages, sb)
    for k, v in T.records.items():
        ref = vals[k]
        err = abs(v.item() - ref)
        if k in pre:   # read a discriminator that Adam already moved
            U = ref - pre[k]
            e = err / max(abs(U), 1e-12)
            ok = err <= TOL_STEP_LOSS * abs(ref) + TOL_STEP_UPDATE * abs(U)
            print('PARITY %s/%-40s got=%.6g ref=%.6g |err|/|U|=%.3e (U=%.4g)' % (tag, k, v.item(), ref, e, U))
        else:
            e = err / max(abs(ref), 1e-3)
            ok = e < TOL_STEP_LOSS
            print('PARITY %s/%-40s got=%.6g ref=%.6g rel=%.3e' % (tag, k, v.item(), ref, e))
        _LOG.append(('%s/%s' % (tag, k), e))
        if os.environ.get('EEGAN_PARITY_SOFT') != '1':   # diagnostics: report every entry, then fail
            assert ok, (k, v.item(), ref)
    # post-Adam parameters: the update is ~lr*sign(g), so compare the parameter
    # CHANGE direction where the reference moved it
    worst = 0.0
    agree = tot = 0
    mods = [('g', G, sb), ('a', A, sb + 1)] + [('d%d' % i, d, sb + 2 + i) for i, d in enumerate(Ds)]
    for nm, mod, seed in mods:
        init = golden_state('%s_%s' % (tag, nm), seed)
        lr = 1e-4 if nm in ('g', 'a') else 4e-4
        for k, v in mod.state_dict().items():
            ref = np.asarray(g['%s/after_%s/%s' % (tag, nm, k)], np.float64).reshape(-1)
            e = _rel_fp(v, ref)
            worst = max(worst, e)
            if os.environ.get('EEGAN_PARITY_SOFT') == '1':
                print('PARAM %s/%s/%s rel %.3e' % (tag, nm, k, e))
            else:
                assert e < 2e-2, (nm, k, e)
            if 'running' in k or 'num_batches' in k:
                continue
            got = np.asarray(fp(v.float().cpu()), np.float64).reshape(-1)
            ini = np.asarray(fp(init[k]), np.float64).reshape(-1)
            off = 6 if ref.size > 4096 or ref.size == 6 + 512 else 0
            dref, dgot = (ref - ini)[off:], (got - ini)[off:]
            sel = np.abs(dref) > 0.5 * lr      # Adam's first steps move each weight by ~lr*sign(grad)
            agree += int((np.sign(dref[sel]) == np.sign(dgot[sel])).sum())
            tot += int(sel.sum())
    frac = agree / max(tot, 1)
    print('PARITY %s/params worst rel_l2 %.3e; Adam-update sign agreement %.4f over %d entries'
          % (tag, worst, frac, tot))
    _LOG.append(('%s/update_sign_agreement' % tag, frac))
    assert frac > TOL_STEP_SIGN


def _graph_vs_eager(gpu, cfg, n_eager, sim_coe=0.05):
    import bench
    from eegan_hip.trainer import StepGraph
    from eegan_hip.synthetic import make_batch
    state, fakes = {}, {}
    for mode in ('eager', 'graph'):
        T, B, ncls = bench.build(cfg, gpu, sim_coe=sim_coe)
        batch = make_batch(B, gpu, seed=11, class_num=ncls, with_class=True)
        noise = seeded_tensor('graph:noise', (B, 100), 1).to(gpu)
        if mode == 'eager':
            for _ in range(n_eager):
                out, _ = T.train_step(batch, noise=noise)
        else:
            sg = StepGraph(T, batch, warmup=1, noise=noise)
            for _ in range(n_eager - 1):
                out, _ = sg.replay()
        torch.cuda.synchronize()
        fakes[mode] = [f.float().cpu() for f in out]
        state[mode] = torch.cat([o.flat for o in [T.optimizerG] + list(T.optimizerDs)] +
                                [o.v for o in [T.optimizerG] + list(T.optimizerDs)])
        del T
        torch.cuda.empty_cache()
    d = (state['graph'] - state['eager']).abs()
    print('STEPGRAPH %s max |graph - eager| over params and Adam moments: %.3e' % (cfg, float(d.max())))
    assert torch.isfinite(state['eager']).all()
    for f in fakes['eager']:
        assert torch.isfinite(f).all() and f.abs().max() <= 1.0   # tanh images
    return state, fakes


def test_step_graph_matches_eager(gpu):
    """The captured step graph (bench.py's execution mode) replays the eager
    step bit for bit, DAMSM included (sim_coe 0.05, the reference default):
    every kernel of the step is deterministic -- the DAMSM region / word
    gradients are fixed-order reductions (csrc/damsm.hip), no atomics."""
    import bench
    from eegan_hip.trainer import StepGraph
    from eegan_hip.synthetic import make_batch
    state = {}
    for mode in ('eager', 'graph'):
        T, B, ncls = bench.build('T8', gpu, sim_coe=0.05)
        batch = make_batch(B, gpu, seed=11, class_num=ncls, with_class=True)
        noise = seeded_tensor('graph:noise', (B, 100), 1).to(gpu)
        if mode == 'eager':
            for _ in range(3):
                T.train_step(batch, noise=noise)
        else:
            sg = StepGraph(T, batch, warmup=1, noise=noise)
            sg.replay()
            sg.replay()
        torch.cuda.synchronize()
        state[mode] = torch.cat([o.flat for o in [T.optimizerG] + list(T.optimizerDs)] +
                                [o.v for o in [T.optimizerG] + list(T.optimizerDs)])
        del T
    d = (state['graph'] - state['eager']).abs()
    print('STEPGRAPH max |graph - eager| over params and Adam moments: %.3e' % float(d.max()))
    assert torch.equal(state['graph'], state['eager'])


@pytest.mark.parametrize('cfg', ['C2', 'C3', 'C4', 'C5'])
def test_config_step_graph_matches_eager(gpu, cfg):
    """Full-size steps of every BASELINE configuration that runs on one GPU:
    C2 (the bench line's workload: CUB, GF=DF=32, batch 16, 200 classes), C3
    (Oxford-102 Flowers, GF=DF=48 -> 48/96/192/384/768 channels on the padded-K
    conv paths, batch 32, 102 classes) and C4's per-GPU shard (MS-COCO,
    GF=DF=64, batch 8, USE_CLASS=False: Dis256 with the DiscSent head) and
    C5's per-GPU shard (CUB, GF=DF=32, 32 images per GPU; its 32 x 256
    global-batch DAMSM block is test_words_block_rectangular's last case).  Size-
    independent properties (the golden fixtures pin the arithmetic at small
    width): finite parameters / moments, images in [-1, 1], and the captured
    step graph equal to the eager step bit for bit."""
    state, fakes = _graph_vs_eager(gpu, cfg, 2)
    assert torch.equal(state['graph'], state['eager'])
    for a, b in zip(fakes['graph'], fakes['eager']):
        assert torch.equal(a, b)


def test_step_deterministic_with_lanes(gpu):
    """The C2 step on its stream lanes is deterministic run to run: three
    fresh trainers from the same seeds end two eager steps with identical
    parameters and Adam moments.  (The generator branch's lane once
    accumulated its first parameter gradients before the main stream's zero
    fill could land -- a race that showed as run-to-run differences only;
    Trainer.zero_grad_G orders the fill before the lane.)"""
    import bench
    from eegan_hip.synthetic import make_batch
    ref = None
    for r in range(3):
        T, B, ncls = bench.build('C2', gpu, sim_coe=0.05)
        assert T.use_streams
        batch = make_batch(B, gpu, seed=11, class_num=ncls, with_class=True)
        noise = seeded_tensor('graph:noise', (B, 100), 1).to(gpu)
        for _ in range(2):
            T.train_step(batch, noise=noise)
        torch.cuda.synchronize()
        st = torch.cat([o.flat for o in [T.optimizerG] + list(T.optimizerDs)] +
                       [o.v for o in [T.optimizerG] + list(T.optimizerDs)])
        if ref is None:
            ref = st
        else:
            print('DETERMINISM run %d max |diff| %.3e' % (r, float((st - ref).abs().max())))
            assert torch.equal(st, ref), r
        del T


def test_damsm_grad_early_trains_attr_enhance(gpu, monkeypatch):
    """The DAMSM branch differentiated on its own lane (trainer.DAMSM_GRAD_EARLY,
    the default) must give ATTR_Enhance the same gradient as the joint
    g_loss.backward() of train.py:493-497: a_loss = sent_loss(cnn_code,
    attrs_emb) (train.py:432) with attrs_emb the trainable ATTR_Enhance output
    (train.py:193-194), so part of ATTR_Enhance's gradient arrives through the
    DAMSM terms, not only through the generator."""
    import models
    from eegan_hip import trainer as TR
    from eegan_hip import functional as Fn
    from sync_batchnorm import DataParallelWithCallback
    from oracle.eegan_oracle import STANDIN_SPEC
    tag = 'step'
    B, W, ncls, disc_class, stages, sb = STEP_CASES[tag]
    grads = {}
    orig_loss = TR.Trainer.DAMSM_loss

    def dropped(self, fake_imgs, sent_emb, words_embs, attrs_emb, *a, **k):   # round 3's bug: no a_loss gradient
        return orig_loss(self, fake_imgs, sent_emb, words_embs, attrs_emb.detach(), *a, **k)
    for early in (True, False, 'dropped'):
        monkeypatch.setattr(TR, 'DAMSM_GRAD_EARLY', bool(early))
        monkeypatch.setattr(TR.Trainer, 'DAMSM_loss', dropped if early == 'dropped' else orig_loss)
        G = _load(models.Gen(W, 100), tag + '_g', sb, gpu)
        A = _load(models.ATTR_Enhance(), tag + '_a', sb + 1, gpu)
        makers = [lambda: models.Dis64(W), lambda: models.Dis128(W), lambda: models.Dis256(W, disc_class, ncls)]
        Ds = [_load(makers[i](), tag + '_d%d' % i, sb + 2 + i, gpu) for i in range(3)]
        standin = _standin_encoder(seeded_state(STANDIN_SPEC, sb + 10), gpu)
        T = TR.Trainer(DataParallelWithCallback(G), DataParallelWithCallback(A),
                       [DataParallelWithCallback(d) for d in Ds], standin, None, B, disc_class=disc_class,
                       class_nums=ncls, class_coe=10.0, sim_coe=0.05, device=gpu)
        batch = synthetic_batch(B, seed=7, class_num=ncls, sizes=(64, 128, 256))
        dbatch = {'imgs': [Fn.ImageToNhwcFn.apply(t.to(gpu)) for t in batch['imgs']],
                  'cls_ids': batch['cls_ids'].to(gpu), 'cap_lens': batch['cap_lens'].to(gpu)}
        emb = tuple(seeded_tensor(tag + ':' + k, shp, 1).to(gpu) for k, shp in
                    (('words', (B, 256, 18)), ('sent', (B, 256)), ('attrs', (B, 3, 256)), ('unpair', (B, 256))))
        T.train_step(dbatch, noise=batch['noise'].to(gpu), emb=emb)
        torch.cuda.synchronize()
        grads[early] = {k: p.grad.detach().float().cpu().clone() for k, p in A.named_parameters()}
    worst = share = 0.0
    for k, g_joint in grads[False].items():
        if k == 'attr_key.bias':   # true gradient identically zero (softmax shift invariance)
            continue
        nrm = g_joint.norm().clamp_min(1e-30)
        worst = max(worst, float((grads[True][k] - g_joint).norm() / nrm))
        share = max(share, float((grads['dropped'][k] - g_joint).norm() / nrm))
    _LOG.append(('damsm_grad_early/attr_enhance worst rel_l2 vs joint backward', worst))
    _LOG.append(('damsm_grad_early/attr_enhance a_loss share (rel_l2 without it)', share))
    print('PARITY damsm_grad_early attr_enhance grads vs joint backward: worst rel_l2 %.3e; without the a_loss '
          'gradient they would differ by %.3e' % (worst, share))
    assert worst < 1e-4, worst
    assert share > 1e-3, share   # the check is sensitive to the dropped term
