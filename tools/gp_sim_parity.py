"""How far does bf16 storage alone move the post-update losses of the golden
whole steps?  (CPU only; tests infrastructure: runs the oracle, never the
product path.)

The GPU test `test_full_step` gates every loss that reads a discriminator
Adam has already moved by |err| <= 3e-2*|ref| + TOL*|U| (U = the update's own
effect on that loss).  This runs the SAME oracle step twice -- fp32, and with
every conv input / output / data gradient rounded to bf16 (oracle.SIM_BF16)
and, with --weights, the conv weights rounded to bf16 as the HIP packs hold
them -- and prints |err|/|U| of the simulated step against the golden values,
i.e. the part of the GPU's figure that bf16 operands alone produce.

  python tools/gp_sim_parity.py [--tags step,stepnc] [--weights]
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, 'tests'))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from _util import golden, golden_state  # noqa: E402
from oracle import eegan_oracle as O  # noqa: E402
from oracle.seeding import seeded_state, seeded_tensor, synthetic_batch  # noqa: E402

STEP_CASES = {'step': (4, 8, 10, True, 3, 50), 'stepnc': (4, 8, 10, False, 3, 110),
              'step12': (2, 12, 10, True, 3, 80), 'step1': (4, 8, 10, True, 1, 90)}


def pre_update(tag):
    B, W, ncls, disc_class, stages, sb = STEP_CASES[tag]
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


def sim_step(tag):
    from oracle.eegan_oracle import STANDIN_SPEC
    B, W, ncls, disc_class, stages, sb = STEP_CASES[tag]
    nd = 3 if stages == 3 else 1
    sd_g, sd_a = golden_state(tag + '_g', sb), golden_state(tag + '_a', sb + 1)
    sd_ds = [golden_state(tag + '_d%d' % i, sb + 2 + i) for i in range(nd)]
    nets = O.OracleNets(sd_g, sd_a, sd_ds, W, W, disc_class, ncls)
    og, ods = O.make_adams(nets)
    sd_enc = seeded_state(STANDIN_SPEC, sb + 10)
    batch = synthetic_batch(B, seed=7, class_num=ncls, sizes=(64, 128, 256))
    emb = tuple(seeded_tensor(tag + ':' + k, s, 1) for k, s in
                (('words', (B, 256, 18)), ('sent', (B, 256)), ('attrs', (B, 3, 256)), ('unpair', (B, 256))))
    _, drec, grec = O.train_step(nets, og, ods, batch, emb, lambda x: O.standin_image_encoder(sd_enc, x),
                                 10.0, 0.05, stages=stages)
    got = {'errD_%d/d_loss_gp' % i: float(gp) for i, (_, gp) in enumerate(drec)}
    got.update({'errG/G_%d_fake_sent' % i: float(e) for i, e in enumerate(grec[1])})
    return got


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--tags', default='step,stepnc')
    ap.add_argument('--weights', action='store_true', help='also round conv weights to bf16')
    args = ap.parse_args()
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    if args.weights:
        def conv_w(x, sd, p, stride=1, pad=0, bias=False):
            w = sd[p + 'weight']
            w = w + (w.detach().to(torch.bfloat16).float() - w.detach())   # straight-through
            return O._r(F.conv2d(O._r(x), w, sd.get(p + 'bias') if bias else None, stride, pad))
        O.conv = conv_w
    g = golden()
    for tag in args.tags.split(','):
        names = json.loads(g[tag + '/scalars/names'].tobytes().decode())
        ref = dict(zip(names, g[tag + '/scalars/values']))
        pre = pre_update(tag)
        res = {}
        for sim in (False, True):
            O.SIM_BF16 = sim
            got = sim_step(tag)
            for k, v in got.items():
                U = ref[k] - pre[k]
                res.setdefault(k, []).append(abs(v - ref[k]) / max(abs(U), 1e-12))
        O.SIM_BF16 = False
        for k in sorted(res):
            print('%s/%-24s |err|/|U|  fp32 oracle %.3e   bf16 sim%s %.3e' % (
                tag, k, res[k][0], ' (+weights)' if args.weights else '', res[k][1]), flush=True)


if __name__ == '__main__':
    main()
