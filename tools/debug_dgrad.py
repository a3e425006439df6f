#!/usr/bin/env python
"""Diagnostic: discriminator parameter gradients of the d_update loss and of
the gradient penalty on the GPU vs the fp32 oracle, on identical inputs (the
oracle's fp32 fake images), for the golden step fixtures.  Prints per-
parameter rel-L2 and gradient sign agreement (entries above 1% of the max)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, 'ee-gan_amd'), os.path.join(REPO, 'tests')):
    sys.path.insert(0, p)

import torch  # noqa: E402


def main(tags):
    import models
    from _util import golden_state, rel_l2
    from oracle import eegan_oracle as O
    from oracle.seeding import synthetic_batch, seeded_tensor
    from eegan_hip import functional as Fn
    from eegan_hip.trainer import Trainer
    from sync_batchnorm import DataParallelWithCallback
    dev = torch.device('cuda', 0)
    cases = {'step': (4, 8, 10, True, 3, 50), 'stepnc': (4, 8, 10, False, 3, 110), 'step12': (2, 12, 10, True, 3, 80)}
    for tag in tags:
        B, W, ncls, dc, stages, sb = cases[tag]
        sd_g, sd_a = golden_state(tag + '_g', sb), golden_state(tag + '_a', sb + 1)
        batch = synthetic_batch(B, seed=7, class_num=ncls, sizes=(64, 128, 256))
        sent = seeded_tensor(tag + ':sent', (B, 256), 1)
        attrs = seeded_tensor(tag + ':attrs', (B, 3, 256), 1)
        unpair = seeded_tensor(tag + ':unpair', (B, 256), 1)
        _, att = O.attr_enhance(sd_a, sent, attrs)
        with torch.no_grad():
            fakes = O.gen_forward(sd_g, batch['noise'], sent, O.attr_merge(att), W)
        for i in range(3):
            mk = [lambda: models.Dis64(W), lambda: models.Dis128(W), lambda: models.Dis256(W, dc, ncls)][i]
            D = mk()
            D.load_state_dict(golden_state(tag + '_d%d' % i, sb + 2 + i))
            D = D.to(dev)
            netD = DataParallelWithCallback(D)
            sd = golden_state(tag + '_d%d' % i, sb + 2 + i)
            for k, v in sd.items():
                if v.is_floating_point() and 'running' not in k:
                    v.requires_grad_(True)
            nets = O.OracleNets({}, {}, [sd] * 3, W, W, dc, ncls)
            real = batch['imgs'][i]
            # oracle d_loss (train.py:437-450)
            rf, ff = nets.d_feat(i, real), nets.d_feat(i, fakes[i])
            if dc and i == 2:
                rs, rc = nets.d_cond(i, rf, sent)
                us, uc = nets.d_cond(i, rf, unpair)
                fs, fc = nets.d_cond(i, ff, sent)
                lab = O.prepare_class_labels(B, ncls, batch['cls_ids'])
                bce = torch.nn.functional.binary_cross_entropy_with_logits
                loss = O.hinge_real(rs) + (O.hinge_fake(fs) + O.hinge_fake(us)) / 2 + \
                    (bce(rc, lab) + bce(fc, lab) + bce(uc, lab)) / 3 * 10
                outs = (rs, us, fs)
            else:
                rs, us, fs = nets.d_cond(i, rf, sent), nets.d_cond(i, rf, unpair), nets.d_cond(i, ff, sent)
                loss = O.hinge_real(rs) + (O.hinge_fake(fs) + O.hinge_fake(us)) / 2
                outs = (rs, us, fs)
            loss.backward()
            print('%s D%d oracle outs real %s unpair %s fake %s' % (tag, i, outs[0].detach().reshape(-1).numpy().round(3),
                                                                  outs[1].detach().reshape(-1).numpy().round(3),
                                                                  outs[2].detach().reshape(-1).numpy().round(3)))
            imgs = Fn.ImageToNhwcFn.apply(real.to(dev))
            fk = Fn.ImageToNhwcFn.apply(fakes[i].to(dev))
            if dc and i == 2:
                labd = Fn.class_onehot(batch['cls_ids'], B, ncls, dev)[0]
                r = Trainer.d_loss_class(imgs, fk, sent.to(dev), unpair.to(dev), labd, netD)
                gl = r[0] + (r[1] + r[2]) / 2 + (r[3] + r[4] + r[5]) / 3 * 10
            else:
                r = Trainer.d_loss(imgs, fk, sent.to(dev), unpair.to(dev), netD)
                gl = r[0] + (r[1] + r[2]) / 2
            D.zero_grad()
            gl.backward()
            print('%s D%d loss gpu %.6g oracle %.6g' % (tag, i, gl.item(), loss.item()))
            bad = []
            for k, p in D.named_parameters():
                if sd[k].grad is None:
                    continue
                gr, gg = sd[k].grad, p.grad.detach().float().cpu()
                sel = gr.abs() > 0.01 * gr.abs().max()
                agree = float((torch.sign(gr[sel]) == torch.sign(gg[sel])).float().mean()) if sel.any() else 1.0
                e = rel_l2(gg, gr)
                bad.append((e, k, agree))
            bad.sort(reverse=True)
            for e, k, a in bad[:6]:
                print('   %-45s rel %.3e sign-agree %.4f' % (k, e, a))


if __name__ == '__main__':
    main(sys.argv[1:] or ['step', 'stepnc'])
