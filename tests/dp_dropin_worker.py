"""The reference train.py's inner step (train.py:186-206, d_update 437-469,
g_update 471-502, the loss statics 336-435) written against the DROP-IN
modules exactly as train.py drives them: Gen wrapped in
DataParallelWithCallback, ATTR_Enhance and the three discriminators in torch's
own nn.DataParallel, torch.optim.Adam(betas=(0, 0.9)) (train.py:252-263),
words_loss / sent_loss from miscc.DAMSM_losses, COND_DNET reached through
`.module`, and NO call into eegan_hip for synchronisation.

Run as one process per rank (torchrun; tests/test_gpu_dist.py launches two
ranks sharing one GPU over gloo) it checks that the drop-in boundary holds at
N > 1: gradient averaging (GradHooks installed by the models' forward),
SyncBN statistics over all ranks and global-batch DAMSM.  Imported without a
process group it is the single-process run of the whole batch.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in (REPO, os.path.join(REPO, 'ee-gan_amd'), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402
import torch.nn.functional as F  # noqa: E402

B_GLOBAL, W, NCLS = 4, 8, 10


def build(dev):
    import models
    from sync_batchnorm import DataParallelWithCallback
    from oracle.seeding import seeded_state, state_spec
    G, A = models.Gen(W, 100), models.ATTR_Enhance()
    Ds = [models.Dis64(W), models.Dis128(W), models.Dis256(W, True, NCLS)]
    for i, m in enumerate([G, A] + Ds):
        m.load_state_dict(seeded_state(state_spec(m.state_dict()), 200 + i))
    netG = DataParallelWithCallback(G.to(dev))
    attr = nn.DataParallel(A.to(dev))
    netsD = [nn.DataParallel(d.to(dev)) for d in Ds]
    optG = torch.optim.Adam(list(netG.parameters()) + list(attr.parameters()), lr=1e-4, betas=(0.0, 0.9))
    optDs = [torch.optim.Adam(d.parameters(), lr=4e-4, betas=(0.0, 0.9)) for d in netsD]
    return netG, attr, netsD, optG, optDs


def standin_encoder(dev):
    from eegan_hip import functional as Fn
    from eegan_hip.nn import Conv2d, Linear
    from oracle.seeding import seeded_state
    from oracle.eegan_oracle import STANDIN_SPEC
    sd = seeded_state(STANDIN_SPEC, 210)
    rconv = Conv2d(3, 256, 15, 15, 0, bias=False).to(dev)
    rconv.weight.data.copy_(sd['standin.regions.weight'].to(dev))
    clin = Linear(256, 256).to(dev)
    clin.weight.data.copy_(sd['standin.code.weight'].to(dev))
    clin.bias.data.copy_(sd['standin.code.bias'].to(dev))
    for p in list(rconv.parameters()) + list(clin.parameters()):
        p.requires_grad_(False)

    def enc(x):
        r = rconv(x, out_f32=True)
        return r, clin(Fn.GlobalAvgPoolFn.apply(Fn.CastF32Bf16Fn.apply(r)))
    return enc


def run_step(rank, world, dev):
    """One iteration on this rank's slice of the global batch; returns the
    logged losses and every parameter after the step."""
    from miscc.DAMSM_losses import words_loss, sent_loss
    from oracle.seeding import synthetic_batch, seeded_tensor
    netG, attr, netsD, optG, optDs = build(dev)
    enc = standin_encoder(dev)
    Bl = B_GLOBAL // world
    sl = slice(rank * Bl, (rank + 1) * Bl)
    batch = synthetic_batch(B_GLOBAL, seed=7, class_num=NCLS, sizes=(64, 128, 256))
    imgs = [t[sl].to(dev) for t in batch['imgs']]
    noise = batch['noise'][sl].to(dev)
    words = seeded_tensor('dp:words', (B_GLOBAL, 256, 18), 1)[sl].to(dev)
    sent = seeded_tensor('dp:sent', (B_GLOBAL, 256), 1)[sl].to(dev)
    attrs = seeded_tensor('dp:attrs', (B_GLOBAL, 3, 256), 1)[sl].to(dev)
    unpair = seeded_tensor('dp:unpair', (B_GLOBAL, 256), 1)[sl].to(dev)
    cap_lens = batch['cap_lens'][sl].to(dev)
    cls_ids = batch['cls_ids'][sl].numpy()
    rec = {}
    # prepare_labels / prepare_class_labels (train.py:90-103)
    match = torch.arange(Bl, device=dev)
    cl = torch.zeros(Bl, NCLS, device=dev)
    for i, idx in enumerate(cls_ids):
        cl[i][int(idx) - 1] = 1
    # train.py:193-195
    _, att = attr(sent, attrs)
    attn_attr = attr.module.attr_merge(att)
    fakes = netG(noise, sent, attn_attr)
    # d_update (train.py:437-469)
    for i, netD in enumerate(netsD):
        real, fake, opt = imgs[i], fakes[i], optDs[i]
        if i == 2:
            rf = netD(real)
            rs, rc = netD.module.COND_DNET(rf, sent)
            us, uc = netD.module.COND_DNET(rf, unpair)
            ff = netD(fake.detach())
            fs, fc = netD.module.COND_DNET(ff, sent)
            bce = F.binary_cross_entropy_with_logits
            e_real, e_un, e_fake = F.relu(1.0 - rs).mean(), F.relu(1.0 + us).mean(), F.relu(1.0 + fs).mean()
            d_loss = e_real + (e_fake + e_un) / 2.0 + (bce(rc, cl) + bce(fc, cl) + bce(uc, cl)) / 3.0 * 10.0
        else:
            rf = netD(real)
            e_real = F.relu(1.0 - netD.module.COND_DNET(rf, sent)).mean()
            e_un = F.relu(1.0 + netD.module.COND_DNET(rf, unpair)).mean()
            e_fake = F.relu(1.0 + netD.module.COND_DNET(netD(fake.detach()), sent)).mean()
            d_loss = e_real + (e_fake + e_un) / 2.0
        opt.zero_grad()
        d_loss.backward()
        opt.step()
        # MA_gradient_penalty (train.py:378-402)
        xi = real.detach().requires_grad_()
        si = sent.detach().requires_grad_()
        out = netD.module.COND_DNET(netD(xi), si)
        if i == 2:
            out = out[0]
        gx, gs = torch.autograd.grad(out, (xi, si), torch.ones_like(out), retain_graph=True, create_graph=True)
        gr = torch.cat((gx.reshape(gx.size(0), -1), gs.reshape(gs.size(0), -1)), 1)
        gp = 2.0 * torch.mean(torch.sqrt(torch.sum(gr ** 2, dim=1)) ** 6)
        opt.zero_grad()
        gp.backward()
        opt.step()
        rec['d%d' % i], rec['gp%d' % i] = float(d_loss), float(gp)
    # g_update (train.py:471-502)
    g_loss = 0
    for i, netD in enumerate(netsD):
        o = netD.module.COND_DNET(netD(fakes[i]), sent)
        if i == 2:
            g_loss = g_loss - o[0].mean() + F.binary_cross_entropy_with_logits(o[1], cl) * 10.0
        else:
            g_loss = g_loss - o.mean()
    regions, code = enc(fakes[-1])
    s0, s1 = sent_loss(code, sent, match, torch.LongTensor(cls_ids), Bl)
    w0, w1, _ = words_loss(regions, words, match, cap_lens, torch.LongTensor(cls_ids), Bl)
    a0, a1 = sent_loss(code, attn_attr, match, torch.LongTensor(cls_ids), Bl)
    g_loss = g_loss + 0.05 * ((s0 + s1) + (w0 + w1) + (a0 + a1))
    optG.zero_grad()
    g_loss.backward()
    optG.step()
    rec.update(s=float(s0 + s1), w=float(w0 + w1), a=float(a0 + a1), g=float(g_loss))
    params = {}
    for nm, m in [('g', netG), ('a', attr)] + [('d%d' % i, d) for i, d in enumerate(netsD)]:
        for k, v in m.module.state_dict().items():
            params['%s/%s' % (nm, k)] = v.detach().float().cpu().clone()
    return rec, params


def main():
    """train.py's process shape under torchrun: the drop-in modules are
    imported first (train.py:22-29), then CUDA_VISIBLE_DEVICES is overwritten
    with the --gpu argument for every rank alike (train.py:513; here '1', i.e.
    `--gpu 1`, a device this one-GPU box does not have), then the device is
    torch.device('cuda') (train.py:114).  No call into torch.distributed or
    eegan_hip.dist: the import pins this rank's GPU and joins the ranks
    (eegan_hip.launch)."""
    import miscc.config  # noqa: F401  (train.py:23-29 import order)
    import miscc.DAMSM_losses  # noqa: F401
    import sync_batchnorm  # noqa: F401
    import models  # noqa: F401
    import DAMSM  # noqa: F401
    os.environ['CUDA_VISIBLE_DEVICES'] = os.environ.get('DP_GPU_IDS', '1')   # train.py:513
    rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
    dev = torch.device('cuda')
    rec, params = run_step(rank, world, dev)
    info = {'device_count': torch.cuda.device_count(), 'rocr': os.environ.get('ROCR_VISIBLE_DEVICES'),
            'hip': os.environ.get('HIP_VISIBLE_DEVICES')}
    torch.save({'rec': rec, 'params': params, 'info': info}, os.path.join(sys.argv[1], 'rank%d.pt' % rank))


if __name__ == '__main__':
    main()
