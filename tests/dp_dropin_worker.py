"""The reference train.py's data + inner step written against the DROP-IN
modules exactly as train.py drives them, with no mention of ranks:

  * imports first (train.py:22-29), then `CUDA_VISIBLE_DEVICES = --gpu`
    (train.py:513), then the seeds (train.py:521-525);
  * `TextDataset` + `torch.utils.data.DataLoader(shuffle=True, drop_last=True)`
    (train.py:265-280) over a small dataset in the reference's on-disk format,
    `prepare_data` (train.py:58-88) with `imgs[i].to(device)`;
  * the networks built from the torch generator in load_networks' order
    (train.py:208-232): Gen in DataParallelWithCallback, ATTR_Enhance and the
    three discriminators in torch's own nn.DataParallel; a frozen text encoder
    (train.py:234-241 loads it from a checkpoint: identical on every rank --
    here seeded weights); torch.optim.Adam(betas=(0, 0.9)) (train.py:252-263);
  * the text encodes (train.py:176-188), `torch.randn(batch_size, 100)`
    (train.py:189), d_update (437-469) and g_update (471-502) with words_loss /
    sent_loss from miscc.DAMSM_losses and COND_DNET through `.module`.

Run as one process per rank (torchrun; tests/test_gpu_dist.py launches two
ranks sharing one GPU over gloo), the drop-in package alone makes this
data-parallel: the import pins and joins the ranks (eegan_hip.launch), the
dataset shards itself and offsets ranks > 0's random streams, the models
broadcast rank 0's weights at their first forward and average gradients with
post-accumulate-grad hooks, SyncBN and DAMSM span the ranks.  Each rank saves
the batch it drew, so the test can step ONE process over the union of the
ranks' batches (`replay`) and compare.
"""
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in (REPO, os.path.join(REPO, 'ee-gan_amd'), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402
import torch.nn.functional as F  # noqa: E402

B_RANK, W, NCLS = 2, 8, 200     # --batch_size (per rank), GF = DF, CLASS_NUM (class_info.pickle holds id 200)
NETS = ('g', 'a', 'd0', 'd1', 'd2')


def build(dev, state=None):
    """load_networks + load_optimizers (train.py:208-263); weights from the
    torch generator as the reference's constructors draw them, or `state`."""
    import models
    from sync_batchnorm import DataParallelWithCallback
    mods = [models.Gen(W, 100), models.ATTR_Enhance(), models.Dis64(W), models.Dis128(W),
            models.Dis256(W, True, NCLS)]
    if state is not None:
        for nm, m in zip(NETS, mods):
            m.load_state_dict(state[nm])
    G, A, Ds = mods[0], mods[1], mods[2:]
    netG = DataParallelWithCallback(G.to(dev))
    attr = nn.DataParallel(A.to(dev))
    netsD = [nn.DataParallel(d.to(dev)) for d in Ds]
    optG = torch.optim.Adam(list(netG.parameters()) + list(attr.parameters()), lr=1e-4, betas=(0.0, 0.9))
    optDs = [torch.optim.Adam(d.parameters(), lr=4e-4, betas=(0.0, 0.9)) for d in netsD]
    return netG, attr, netsD, optG, optDs


def encoders(dev, n_words):
    """The frozen text encoder (seeded: the checkpoint of train.py:236 is the
    same file on every rank) and a small stand-in image encoder for DAMSM."""
    import DAMSM
    from eegan_hip import functional as Fn
    from eegan_hip.nn import Conv2d, Linear
    from oracle.seeding import seeded_state, state_spec
    from oracle.eegan_oracle import STANDIN_SPEC
    text = DAMSM.RNN_ENCODER(n_words, nhidden=256)
    text.load_state_dict(seeded_state(state_spec(text.state_dict()), 211))
    text = text.to(dev).eval()
    for p in text.parameters():
        p.requires_grad = False
    sd = seeded_state(STANDIN_SPEC, 210)
    rconv = Conv2d(3, 256, 15, 15, 0, bias=False).to(dev)
    rconv.weight.data.copy_(sd['standin.regions.weight'].to(dev))
    clin = Linear(256, 256).to(dev)
    clin.weight.data.copy_(sd['standin.code.weight'].to(dev))
    clin.bias.data.copy_(sd['standin.code.bias'].to(dev))
    for p in list(rconv.parameters()) + list(clin.parameters()):
        p.requires_grad_(False)

    def image(x):
        r = rconv(x, out_f32=True)
        return r, clin(Fn.GlobalAvgPoolFn.apply(Fn.CastF32Bf16Fn.apply(r)))
    return text, image


def prepare_data(data, device):
    """train.py:58-88."""
    rev_basic, rev_attrs, rev_unpair = data
    imgs, caps, cap_lens, cls_ids, keys = rev_basic
    attrs, attr_nums, attrs_len = rev_attrs
    unpair_caps, unpair_cap_lens, unpair_cls_ids = rev_unpair
    real_imgs = [imgs[i].to(device) for i in range(len(imgs))]
    return {'imgs': real_imgs, 'caps': caps.squeeze().to(device), 'cap_lens': cap_lens.to(device),
            'cls_ids': cls_ids.numpy(), 'attrs': attrs.squeeze().to(device), 'attrs_len': attrs_len.squeeze(),
            'unpair_caps': unpair_caps.squeeze().to(device), 'unpair_cap_lens': unpair_cap_lens.to(device),
            'keys': list(keys)}


def encode(text, b, B):
    """train.py:176-188."""
    with torch.no_grad():
        hidden = text.init_hidden(B)
        words, sent = text(b['caps'], b['cap_lens'], hidden)
        ae = []
        for i in range(b['attrs'].shape[1]):
            _, e = text(b['attrs'][:, i, :].squeeze(-1), b['attrs_len'][:, i].squeeze(-1), hidden)
            ae.append(e)
        attrs_emb = torch.stack(ae, dim=1)
        _, unpair = text(b['unpair_caps'], b['unpair_cap_lens'], hidden)
    return words.detach(), sent.detach(), attrs_emb.detach(), unpair.detach()


def step(nets, image_enc, b, words, sent, attrs_emb, unpair, noise, B, dev):
    """train.py:186-206 with d_update (437-469) and g_update (471-502);
    returns the logged losses."""
    from miscc.DAMSM_losses import words_loss, sent_loss
    netG, attr, netsD, optG, optDs = nets
    imgs, cap_lens, cls_ids = b['imgs'], b['cap_lens'], b['cls_ids']
    rec = {}
    # prepare_labels / prepare_class_labels (train.py:90-103)
    match = torch.arange(B, device=dev)
    cl = torch.zeros(B, NCLS, device=dev)
    for i, idx in enumerate(cls_ids):
        cl[i][int(idx) - 1] = 1
    # train.py:193-195
    _, att = attr(sent, attrs_emb)
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
    regions, code = image_enc(fakes[-1])
    cids = torch.LongTensor(np.asarray(cls_ids, dtype=np.int64))
    s0, s1 = sent_loss(code, sent, match, cids, B)
    w0, w1, _ = words_loss(regions, words, match, cap_lens, cids, B)
    a0, a1 = sent_loss(code, attn_attr, match, cids, B)
    g_loss = g_loss + 0.05 * ((s0 + s1) + (w0 + w1) + (a0 + a1))
    optG.zero_grad()
    g_loss.backward()
    optG.step()
    rec.update(s=float(s0 + s1), w=float(w0 + w1), a=float(a0 + a1), g=float(g_loss))
    return rec


def states(nets):
    netG, attr, netsD = nets[:3]
    out = {}
    for nm, m in zip(NETS, [netG, attr] + list(netsD)):
        out[nm] = {k: v.detach().cpu().clone() for k, v in m.module.state_dict().items()}
    return out


def flat_params(st):
    return {'%s/%s' % (nm, k): v.float() for nm in NETS for k, v in st[nm].items()}


def replay(records, dev, n_words):
    """ONE process stepping the union of the ranks' batches (rank order), from
    rank 0's initial weights: the reference's single-process DataParallel
    step over the whole batch."""
    nets = build(dev, records[0]['init'])
    text, image = encoders(dev, n_words)
    cat = lambda k: torch.cat([r['batch'][k] for r in records], 0)  # noqa: E731
    b = {'imgs': [torch.cat([r['batch']['imgs'][s] for r in records], 0).to(dev) for s in range(3)],
         'caps': cat('caps').to(dev), 'cap_lens': cat('cap_lens').to(dev),
         'cls_ids': cat('cls_ids').numpy(),
         'attrs': cat('attrs').to(dev), 'attrs_len': cat('attrs_len'),
         'unpair_caps': cat('unpair_caps').to(dev), 'unpair_cap_lens': cat('unpair_cap_lens').to(dev)}
    B = len(b['cls_ids'])
    words, sent, attrs_emb, unpair = encode(text, b, B)
    rec = step(nets, image, b, words, sent, attrs_emb, unpair, cat('noise').to(dev), B, dev)
    return rec, flat_params(states(nets))


def main(data_dir, out):
    """train.py's process shape under torchrun, in train.py's order."""
    import miscc.config  # noqa: F401  (train.py:22-29 import order)
    import miscc.DAMSM_losses  # noqa: F401
    import sync_batchnorm  # noqa: F401
    from datasets import TextDataset
    import models  # noqa: F401
    import DAMSM  # noqa: F401
    os.environ['CUDA_VISIBLE_DEVICES'] = os.environ.get('DP_GPU_IDS', '1')   # train.py:513 (`--gpu 1`)
    random.seed(3407)                                                       # train.py:521-525
    np.random.seed(3407)
    torch.manual_seed(3407)
    dev = torch.device('cuda')                                              # train.py:114
    ds = TextDataset(data_dir=data_dir, dataset_name='bird', transform=None)
    loader = torch.utils.data.DataLoader(ds, batch_size=B_RANK, drop_last=True, shuffle=True, num_workers=0)
    nets = build(dev)
    init = states(nets)
    text, image = encoders(dev, ds.n_words)
    b = prepare_data(next(iter(loader)), dev)
    words, sent, attrs_emb, unpair = encode(text, b, B_RANK)
    noise = torch.randn(B_RANK, 100)                                        # train.py:189
    batch = {'imgs': [t.cpu() for t in b['imgs']], 'noise': noise.clone(), 'keys': b['keys'],
             'cls_ids': torch.as_tensor(np.asarray(b['cls_ids'], dtype=np.int64)), 'attrs_len': b['attrs_len'].clone()}
    for k in ('caps', 'cap_lens', 'attrs', 'unpair_caps', 'unpair_cap_lens'):
        batch[k] = b[k].cpu()
    rec = step(nets, image, b, words, sent, attrs_emb, unpair, noise.to(dev), B_RANK, dev)
    info = {'device_count': torch.cuda.device_count(), 'rocr': os.environ.get('ROCR_VISIBLE_DEVICES'),
            'hip': os.environ.get('HIP_VISIBLE_DEVICES'), 'len': len(ds), 'n_words': ds.n_words,
            'base': [ds.base_index(i) for i in range(len(ds))]}
    torch.save({'rec': rec, 'params': flat_params(states(nets)), 'init': init, 'batch': batch, 'info': info},
               os.path.join(out, 'rank%s.pt' % os.environ['RANK']))


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
