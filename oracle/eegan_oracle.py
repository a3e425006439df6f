"""CPU oracle: a functional fp32 restatement of EE-GAN's data-parallel G+D
training step (the hot path of BASELINE.json's north_star).

TEST INFRASTRUCTURE ONLY -- imported by tests/, bench.py's ``cpu_baseline``
leg, __graft_entry__.smoke() and the golden-fixture script.  The product
(``ee-gan_amd/``) never imports it.

Pinning: every function here is checked against golden vectors produced by
importing the reference itself in the build container
(tests/golden/make_golden.py -> tests/golden/*.npz, tests/test_oracle_golden.py).
The Inception-v3 image encoder (``inception_*``) cannot be pinned that way
(torchvision is absent, DAMSM.py:14,127) -- it is restated from torchvision's
published ``inception_v3`` definition and is marked *parity unpinned*.

Parameters are passed as a flat ``sd`` dict keyed exactly like the
reference's ``state_dict()`` (models.py / DAMSM.py); BatchNorm running
buffers in ``sd`` are updated in place exactly like ``F.batch_norm`` does.
"""
import math

import torch
import torch.nn.functional as F

# hyper-parameters of miscc/config.py:47-51
GAMMA1, GAMMA2, GAMMA3, LAMBDA = 5.0, 5.0, 10.0, 1.0
BN_EPS, BN_MOM = 1e-5, 0.1


# --------------------------------------------------------------------------
# SyncBN (sync_batchnorm/batchnorm.py:48-125)
# --------------------------------------------------------------------------
def sync_bn(x, sd, p, affine=True, training=True, mode='single'):
    """``mode='single'``: 1 device / CPU path -> F.batch_norm (batchnorm.py:50-53).
    ``mode='multi'``: the cross-replica formula of batchnorm.py:57-75,113-125
    (clamp(var_biased, eps)^-1/2, running_var from the unbiased variance),
    restated for one process holding the whole (global) batch."""
    w = sd.get(p + 'weight') if affine else None
    b = sd.get(p + 'bias') if affine else None
    if mode == 'single' or not training:
        return F.batch_norm(x, sd[p + 'running_mean'], sd[p + 'running_var'], w, b,
                            training, BN_MOM, BN_EPS)
    C = x.shape[1]
    xv = x.reshape(x.shape[0], C, -1)
    n = xv.shape[0] * xv.shape[2]
    s = xv.sum(dim=0).sum(dim=-1)
    ss = (xv ** 2).sum(dim=0).sum(dim=-1)
    mean = s / n
    sumvar = ss - s * mean
    with torch.no_grad():
        sd[p + 'running_mean'].mul_(1 - BN_MOM).add_(BN_MOM * mean.detach())
        sd[p + 'running_var'].mul_(1 - BN_MOM).add_(BN_MOM * (sumvar / (n - 1)).detach())
    inv_std = (sumvar / n).clamp(BN_EPS) ** -0.5
    y = (xv - mean[None, :, None]) * inv_std[None, :, None]
    if affine:
        y = y * w[None, :, None] + b[None, :, None]
    return y.reshape(x.shape)


class _RoundBF16(torch.autograd.Function):
    """Straight-through bf16 rounding of an activation (forward) and of the
    gradient flowing back through it (backward)."""

    @staticmethod
    def forward(ctx, x):
        return x.to(torch.bfloat16).to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).to(g.dtype)


# bf16 SIMULATION switch (tests only): when True every conv input and output
# -- the activations and data gradients the HIP path stores as bf16 -- is
# rounded to bf16, so the fp32 oracle measures how far bf16 storage alone
# moves a result from the reference (the basis of the deep-gradient gates in
# tests/test_gpu_models.py).  Off by default: the oracle is the fp32 reference.
SIM_BF16 = False


def _r(x):
    return _RoundBF16.apply(x) if SIM_BF16 else x


# gain-gradient PROBE (tests only): when a dict, every residual gain
# out = shortcut + gamma * h records (h, out) under its parameter prefix, so a
# test can form the Cauchy-Schwarz scale ||d out|| * ||h|| that bounds how far
# d gamma = <d out, h> moves when d out carries a relative error.
PROBE = None


def _probe(p, h, out):
    if PROBE is not None:
        if out.requires_grad:
            out.retain_grad()
        PROBE[p] = (h, out)


def linear(x, sd, p, bias=True):
    return F.linear(x, sd[p + 'weight'], sd[p + 'bias'] if bias else None)


def conv(x, sd, p, stride=1, pad=0, bias=False):
    return _r(F.conv2d(_r(x), sd[p + 'weight'], sd.get(p + 'bias') if bias else None, stride, pad))


# --------------------------------------------------------------------------
# Generator side (models.py:25-256)
# --------------------------------------------------------------------------
def mask_head(sd, p, x, bn_mode='single'):
    """get_mask: conv3x3 -> BN(100) -> ReLU -> conv1x1 (models.py:34-41)."""
    h = conv(x, sd, p + '0.', 1, 1)
    h = F.relu(sync_bn(h, sd, p + '1.', True, mode=bn_mode))
    return conv(h, sd, p + '3.')


def image_head(sd, p, x, bn_mode='single'):
    """get_image: BN -> LeakyReLU(0.2) -> conv3x3 -> tanh (models.py:25-32)."""
    h = F.leaky_relu(sync_bn(x, sd, p + '0.', True, mode=bn_mode), 0.2)
    return torch.tanh(conv(h, sd, p + '2.', 1, 1))


def affine_ssa(sd, p, feat, cond, smask, bn_mode='single'):
    """models.py:69-86: n = BN_noaffine(feat); out = (gamma*m + 1)*n + beta*m,
    gamma/beta = Linear->ReLU->Linear(cond)."""
    n = sync_bn(feat, sd, p + 'norm2d.', affine=False, mode=bn_mode)
    g = linear(F.relu(linear(cond, sd, p + 'fc_gamma.linear1.')), sd, p + 'fc_gamma.linear2.')
    b = linear(F.relu(linear(cond, sd, p + 'fc_beta.linear1.')), sd, p + 'fc_beta.linear2.')
    if g.dim() == 1:
        g = g.unsqueeze(0)
    if b.dim() == 1:
        b = b.unsqueeze(0)
    g = g[:, :, None, None]
    b = b[:, :, None, None]
    return (g * smask + 1) * n + b * smask


def sagb_block(sd, p, feat, conds, smask, learnable_sc, pred_mask, bn_mode='single'):
    """SAGB_Block.forward (models.py:108-126)."""
    sc = conv(feat, sd, p + 'c_sc.', bias=True) if learnable_sc else feat
    h = F.relu(affine_ssa(sd, p + 'affine1.', feat, conds[0], smask, bn_mode))
    h = conv(h, sd, p + 'c1.', 1, 1)
    h = F.relu(affine_ssa(sd, p + 'affine2.', h, conds[1], smask, bn_mode))
    h = conv(h, sd, p + 'c2.', 1, 1)
    out = _r(sc + sd[p + 'gamma'] * h)
    _probe(p, h, out)
    m = mask_head(sd, p + 'conv_mask.', out, bn_mode) if pred_mask else None
    return out, m


def cum_block(sd, p, prev, cur):
    """Cum_Block.forward (models.py:140-143)."""
    u = conv(prev, sd, p + 'up_block.0.')
    u = F.interpolate(u, scale_factor=2, mode='nearest')
    u = conv(u, sd, p + 'up_block.2.', 1, 1)
    s = u + cur * sd[p + 'gamma']
    _probe(p, cur, s)
    return conv(s, sd, p + 'fuse_block.', 1, 1)


def gen_channels(ngf):
    """(in, out, pred_mask) of Gen.blocks (models.py:189-204)."""
    return [(8 * ngf, 8 * ngf, True)] * 4 + [(8 * ngf, 4 * ngf, True), (4 * ngf, 2 * ngf, True),
                                              (2 * ngf, ngf, False)]


def gen_forward(sd, z, sent, attrs, ngf, bn_mode='single', stages=3):
    """Gen.forward (models.py:225-256). ``stages=1`` is the harness-defined
    stage-1 slice of config C1: up to img_64 only."""
    chans = gen_channels(ngf)
    B = z.shape[0]
    out = _r(linear(z, sd, 'fc.').view(B, 8 * ngf, 4, 4))
    m = mask_head(sd, 'init_mask.', out, bn_mode)
    out, m = sagb_block(sd, 'blocks.0.', out, (sent, sent), torch.sigmoid(m),
                        chans[0][0] != chans[0][1], chans[0][2], bn_mode)

    def progress(x, conds, m, scale, ix):
        x = F.interpolate(x, scale_factor=2)
        m = torch.sigmoid(F.interpolate(m, size=scale, mode='bilinear', align_corners=True))
        cin, cout, pm = chans[ix]
        return sagb_block(sd, 'blocks.%d.' % ix, x, conds, m, cin != cout, pm, bn_mode)

    for ix, scale in enumerate([8, 16, 32]):
        out, m = progress(out, (sent, sent), m, scale, ix + 1)
    x32 = out
    x64, m = progress(x32, (sent, attrs), m, 64, 4)
    c64 = cum_block(sd, 'cum_64.', x32, x64)
    img64 = image_head(sd, 'get_image_64.', c64, bn_mode)
    if stages == 1:
        return [img64]
    x128, m = progress(x64, (sent, attrs), m, 128, 5)
    x256, _ = progress(x128, (sent, attrs), m, 256, 6)
    c128 = cum_block(sd, 'cum_128.', c64, x128)
    c256 = cum_block(sd, 'cum_256.', c128, x256)
    img128 = image_head(sd, 'get_image_128.', c128, bn_mode)
    img256 = image_head(sd, 'get_image_256.', c256, bn_mode)
    return [img64, img128, img256]


def attr_enhance(sd, sent, attrs, p=''):
    """ATTR_Enhance.forward (models.py:155-169); softmax THEN x 1/sqrt(ntf)."""
    x = torch.cat([sent.unsqueeze(1), attrs], dim=1)
    q = linear(x, sd, p + 'attr_query.')
    k = linear(x, sd, p + 'attr_key.')
    v = linear(x, sd, p + 'attr_value.')
    a = torch.softmax(torch.bmm(q, k.transpose(1, 2)), dim=-1) * (1.0 / math.sqrt(x.shape[-1]))
    out = torch.bmm(a, v)
    return out[:, 0, :], out


def attr_merge(attn_attrs):
    """ATTR_Enhance.attr_merge (models.py:172-180): sum over the 4 rows."""
    return attn_attrs.sum(dim=1)


# --------------------------------------------------------------------------
# Discriminator side (models.py:262-403)
# --------------------------------------------------------------------------
def res_d(sd, p, x, fin, fout):
    """resD.forward (models.py:277-288)."""
    r = F.leaky_relu(conv(x, sd, p + 'conv_r.0.', 2, 1), 0.2)
    r = F.leaky_relu(conv(r, sd, p + 'conv_r.2.', 1, 1), 0.2)
    s = conv(x, sd, p + 'conv_s.', bias=True) if fin != fout else x
    s = F.avg_pool2d(s, 2)
    return s + sd[p + 'gamma'] * r


def dis_channels(kind, ndf):
    m = {64: [1, 2, 4, 8, 8], 128: [1, 2, 4, 8, 8, 16], 256: [1, 2, 4, 8, 16, 16, 16]}[kind]
    return [(ndf * a, ndf * b) for a, b in zip(m[:-1], m[1:])]


def dis_forward(sd, x, kind, ndf):
    """Dis64/128/256.forward (models.py:350-403)."""
    h = conv(x, sd, 'conv_img.', 1, 1, bias=True)
    for i, (fi, fo) in enumerate(dis_channels(kind, ndf)):
        h = res_d(sd, 'block%d.' % i, h, fi, fo)
    return h


def disc_sent(sd, feat, cond, p='COND_DNET.'):
    """DiscSent.forward (models.py:301-306)."""
    c = cond.reshape(-1, cond.shape[-1], 1, 1).repeat(1, 1, 4, 4)
    h = torch.cat((feat, c), 1)
    h = F.leaky_relu(conv(h, sd, p + 'joint_conv.0.', 1, 1), 0.2)
    return conv(h, sd, p + 'joint_conv.2.')


def disc_cond(sd, feat, cond, p='COND_DNET.'):
    """DiscCond.forward (models.py:323-338) -> (pair (B,), class logits)."""
    s = feat.shape[-1]
    c = cond.reshape(-1, cond.shape[-1], 1, 1).repeat(1, 1, s, s)
    h = torch.cat((feat, c), 1)
    h = F.leaky_relu(conv(h, sd, p + 'joinConv.0.', 1, 1), 0.2)
    pair = F.conv2d(h, sd[p + 'pair_node.weight'], sd[p + 'pair_node.bias'], 4).view(-1)
    cls = F.conv2d(h, sd[p + 'class_node.weight'], sd[p + 'class_node.bias'], 4)
    cls = cls.view(-1, sd[p + 'class_node.weight'].shape[0])
    return pair, linear(cls, sd, p + 'class_linear.')


# --------------------------------------------------------------------------
# DAMSM losses (miscc/DAMSM_losses.py)
# --------------------------------------------------------------------------
def cosine_similarity(x1, x2, dim=1, eps=1e-8):
    """DAMSM_losses.py:17-23."""
    w12 = (x1 * x2).sum(dim)
    return (w12 / (x1.norm(2, dim) * x2.norm(2, dim)).clamp(min=eps)).squeeze()


def func_attention(query, context, gamma1):
    """DAMSM_losses.py:25-63. query (B,D,L); context (B,D,ih,iw)."""
    B, L = query.shape[0], query.shape[2]
    ih, iw = context.shape[2], context.shape[3]
    ctx = context.reshape(B, -1, ih * iw)
    s = torch.bmm(ctx.transpose(1, 2), query)                    # B x R x L
    a = torch.softmax(s.reshape(B * ih * iw, L), dim=1).reshape(B, ih * iw, L)
    a = a.transpose(1, 2).reshape(B * L, ih * iw)
    a = torch.softmax(a * gamma1, dim=1).reshape(B, L, ih * iw)
    wc = torch.bmm(ctx, a.transpose(1, 2))                       # B x D x L
    return wc, a.reshape(B, -1, ih, iw)


def _class_mask(class_ids, B):
    """same-class off-diagonal mask (DAMSM_losses.py:238-243, 282-285)."""
    if class_ids is None:
        return None
    cid = torch.as_tensor(class_ids).reshape(-1)
    m = cid[None, :] == cid[:B, None]
    m = m.clone()
    m[torch.arange(B), torch.arange(B)] = False
    return m


def sent_loss(cnn_code, rnn_code, labels, class_ids, batch_size, eps=1e-8):
    """DAMSM_losses.py:233-270."""
    mask = _class_mask(class_ids, batch_size)
    num = cnn_code @ rnn_code.t()
    den = cnn_code.norm(2, dim=1, keepdim=True) @ rnn_code.norm(2, dim=1, keepdim=True).t()
    s0 = num / den.clamp(min=eps) * GAMMA3
    if mask is not None:
        s0 = s0.masked_fill(mask, -float('inf'))
    if labels is None:
        return None, None
    return F.cross_entropy(s0, labels), F.cross_entropy(s0.t(), labels)


def words_similarity_matrix(img_features, words_emb, cap_lens, class_ids, batch_size):
    """The (image j, text i) matrix of DAMSM_losses.py:281-333 (x gamma3, masked)."""
    lens = [int(v) for v in torch.as_tensor(cap_lens).reshape(-1).tolist()]
    cols, maps = [], []
    for i in range(batch_size):
        w = lens[i]
        word = words_emb[i, :, :w].unsqueeze(0).expand(batch_size, -1, -1)
        wc, attn = func_attention(word, img_features, GAMMA1)
        maps.append(attn[i].unsqueeze(0))
        cos = cosine_similarity(word.transpose(1, 2).reshape(batch_size * w, -1),
                                wc.transpose(1, 2).reshape(batch_size * w, -1))
        r = torch.exp(cos.reshape(batch_size, w) * GAMMA2).sum(dim=1, keepdim=True)
        cols.append(torch.log(r))
    sim = torch.cat(cols, 1) * GAMMA3
    mask = _class_mask(class_ids, batch_size)
    if mask is not None:
        sim = sim.masked_fill(mask, -float('inf'))
    return sim, maps


def words_loss(img_features, words_emb, labels, cap_lens, class_ids, batch_size):
    """DAMSM_losses.py:272-342."""
    sim, maps = words_similarity_matrix(img_features, words_emb, cap_lens, class_ids, batch_size)
    if labels is None:
        return None, None, maps
    return F.cross_entropy(sim, labels), F.cross_entropy(sim.t(), labels), maps


def global_attention_general(inp, context_key, content_value, mask=None):
    """GlobalAttentionGeneral.forward (DAMSM_losses.py:75-132)."""
    B, _, ih, iw = inp.shape
    Lq = ih * iw
    S = context_key.shape[2]
    a = torch.bmm(inp.reshape(B, -1, Lq).transpose(1, 2), context_key).reshape(B * Lq, S)
    if mask is not None:
        a = a.masked_fill(mask.repeat(Lq, 1), -float('inf'))
    a = torch.softmax(a, dim=1).reshape(B, Lq, S).transpose(1, 2)
    wc = torch.bmm(content_value, a)
    return wc.reshape(B, -1, ih, iw), a.reshape(B, -1, ih, iw)


# --------------------------------------------------------------------------
# train.py statics (train.py:90-103, 336-435)
# --------------------------------------------------------------------------
def prepare_labels(B):
    return torch.ones(B), torch.zeros(B), torch.arange(B)


def prepare_class_labels(B, class_num, class_ids):
    """train.py:99-103 -- note ``idx - 1`` wraps id 0 to column class_num-1."""
    lab = torch.zeros(B, class_num)
    for i, idx in enumerate(class_ids):
        lab[i][int(idx) - 1] = 1
    return lab


def hinge_real(o):
    return F.relu(1.0 - o).mean()


def hinge_fake(o):
    return F.relu(1.0 + o).mean()


def gradient_penalty(grad_img, grad_sent):
    """MA_gradient_penalty tail (train.py:396-402)."""
    g = torch.cat((grad_img.reshape(grad_img.shape[0], -1), grad_sent.reshape(grad_sent.shape[0], -1)), 1)
    return 2.0 * torch.mean(torch.sqrt((g ** 2).sum(1)) ** 6)


class OracleNets:
    """Bundles the state dicts of G, ATTR_Enhance and the 3 D's."""

    def __init__(self, sd_g, sd_a, sd_ds, ngf, ndf, disc_class, class_nums, bn_mode='single'):
        self.sd_g, self.sd_a, self.sd_ds = sd_g, sd_a, sd_ds
        self.ngf, self.ndf, self.disc_class, self.class_nums = ngf, ndf, disc_class, class_nums
        self.bn_mode = bn_mode
        for sd in [sd_g, sd_a] + list(sd_ds):
            for k, v in sd.items():
                if v.is_floating_point() and not ('running' in k):
                    v.requires_grad_(True)

    def d_feat(self, i, x):
        return dis_forward(self.sd_ds[i], x, [64, 128, 256][i], self.ndf)

    def d_cond(self, i, feat, cond):
        if i == 2 and self.disc_class:
            return disc_cond(self.sd_ds[i], feat, cond)
        return disc_sent(self.sd_ds[i], feat, cond)

    def params(self, sd):
        return [v for k, v in sd.items() if v.is_floating_point() and 'running' not in k]


def make_adams(nets, lr_g=1e-4, lr_d=4e-4):
    """train.py:252-263."""
    og = torch.optim.Adam(nets.params(nets.sd_g) + nets.params(nets.sd_a), lr=lr_g, betas=(0.0, 0.9))
    ods = [torch.optim.Adam(nets.params(sd), lr=lr_d, betas=(0.0, 0.9)) for sd in nets.sd_ds]
    return og, ods


def d_update(nets, opts_d, imgs, fakes, sent, unpair, class_labels, class_coe, n_d=3):
    """train.py:437-459 incl. MA_gradient_penalty (378-402): per D one hinge
    (+class BCE) step and one gradient-penalty step."""
    rec = []
    for i in range(n_d):
        dc = nets.disc_class and i == 2
        real_f = nets.d_feat(i, imgs[i])
        fake_f = nets.d_feat(i, fakes[i].detach())
        if dc:
            rs, rc = nets.d_cond(i, real_f, sent)
            us, uc = nets.d_cond(i, real_f, unpair)
            fs, fc = nets.d_cond(i, fake_f, sent)
            e_real, e_un, e_fake = hinge_real(rs), hinge_fake(us), hinge_fake(fs)
            bce = F.binary_cross_entropy_with_logits
            cl = (bce(rc, class_labels) + bce(fc, class_labels) + bce(uc, class_labels)) / 3.0
            loss = e_real + (e_fake + e_un) / 2.0 + cl * class_coe
        else:
            e_real = hinge_real(nets.d_cond(i, real_f, sent))
            e_un = hinge_fake(nets.d_cond(i, real_f, unpair))
            e_fake = hinge_fake(nets.d_cond(i, fake_f, sent))
            loss = e_real + (e_fake + e_un) / 2.0
        opts_d[i].zero_grad()
        loss.backward()
        opts_d[i].step()
        xi = imgs[i].detach().requires_grad_()
        si = sent.detach().requires_grad_()
        out = nets.d_cond(i, nets.d_feat(i, xi), si)
        if dc:
            out = out[0]
        gx, gs = torch.autograd.grad(out, (xi, si), torch.ones_like(out), retain_graph=True,
                                     create_graph=True)
        gp = gradient_penalty(gx, gs)
        opts_d[i].zero_grad()
        gp.backward()
        opts_d[i].step()
        rec.append((loss.detach(), gp.detach()))
    return rec


def g_update(nets, opt_g, fakes, sent, words, attr_emb, class_ids, match_labels, cap_lens,
             class_labels, class_coe, sim_coe, image_encoder, n_d=3):
    """train.py:471-502 with DAMSM_loss (419-435)."""
    B = sent.shape[0]
    g_loss = torch.zeros(1)
    errs = []
    for i in range(n_d):
        f = nets.d_feat(i, fakes[i])
        if nets.disc_class and i == 2:
            s, c = nets.d_cond(i, f, sent)
            e = -s.mean()
            g_loss = g_loss + e + F.binary_cross_entropy_with_logits(c, class_labels) * class_coe
        else:
            e = -nets.d_cond(i, f, sent).mean()
            g_loss = g_loss + e
        errs.append(e.detach())
    cids = torch.as_tensor(class_ids)
    regions, code = image_encoder(fakes[-1])
    s0, s1 = sent_loss(code, sent, match_labels, cids, B)
    w0, w1, _ = words_loss(regions, words, match_labels, cap_lens, cids, B)
    a0, a1 = sent_loss(code, attr_emb, match_labels, cids, B)
    damsm = ((w0 + w1) * LAMBDA, (s0 + s1) * LAMBDA, (a0 + a1) * LAMBDA)
    g_loss = g_loss + sim_coe * (damsm[1] + damsm[0] + damsm[2])
    opt_g.zero_grad()
    g_loss.backward()
    opt_g.step()
    return g_loss.detach(), errs, [d.detach() for d in damsm]


def train_step(nets, opt_g, opts_d, batch, emb, image_encoder, class_coe=10.0, sim_coe=0.05,
               stages=3):
    """One iteration of train.py:186-206 given precomputed text embeddings
    ``emb = (words_emb, sent_emb, attrs_emb(B,3,256), unpair_sent_emb)``."""
    words, sent, attrs, unpair = emb
    B = sent.shape[0]
    class_labels = None
    if nets.disc_class:
        class_labels = prepare_class_labels(B, nets.class_nums, batch['cls_ids'])
    _, att = attr_enhance(nets.sd_a, sent, attrs)
    attn_attr = attr_merge(att)
    fakes = gen_forward(nets.sd_g, batch['noise'], sent, attn_attr, nets.ngf, nets.bn_mode, stages)
    n_d = 3 if stages == 3 else 1
    drec = d_update(nets, opts_d, batch['imgs'], fakes, sent, unpair, class_labels, class_coe, n_d)
    _, _, match = prepare_labels(B)
    grec = g_update(nets, opt_g, fakes, sent, words, attn_attr, batch['cls_ids'], match,
                    batch['cap_lens'], class_labels, class_coe, sim_coe, image_encoder, n_d)
    return fakes, drec, grec


# --------------------------------------------------------------------------
# Frozen encoders (DAMSM.py) -- "next" rows of SURVEY.md §8(f)
# --------------------------------------------------------------------------
def rnn_encoder(sd, captions, cap_lens, nhidden=256):
    """RNN_ENCODER.forward (DAMSM.py:88-115) in eval mode: embedding ->
    bi-LSTM over each sequence's own length; words (B,nhidden,T_max),
    sent = [h_fwd(last valid), h_bwd(first)] (B,nhidden)."""
    emb = F.embedding(captions, sd['encoder.weight'])
    B, T, _ = emb.shape
    H = nhidden // 2
    lens = torch.as_tensor(cap_lens).reshape(-1).tolist()
    Tm = int(max(lens))
    out = torch.zeros(B, Tm, 2 * H)
    hlast = torch.zeros(2, B, H)
    for d, sfx in enumerate(['', '_reverse']):
        Wih, Whh = sd['rnn.weight_ih_l0' + sfx], sd['rnn.weight_hh_l0' + sfx]
        bias = sd['rnn.bias_ih_l0' + sfx] + sd['rnn.bias_hh_l0' + sfx]
        for b in range(B):
            L = int(lens[b])
            h = torch.zeros(H)
            c = torch.zeros(H)
            steps = range(L) if d == 0 else range(L - 1, -1, -1)
            for t in steps:
                gates = Wih @ emb[b, t] + Whh @ h + bias
                i_, f_, g_, o_ = gates.split(H)
                c = torch.sigmoid(f_) * c + torch.sigmoid(i_) * torch.tanh(g_)
                h = torch.sigmoid(o_) * torch.tanh(c)
                out[b, t, d * H:(d + 1) * H] = h
            hlast[d, b] = h
    words = out.transpose(1, 2)
    sent = hlast.transpose(0, 1).reshape(B, 2 * H)
    return words, sent


def _basic_conv(sd, p, x, stride=1, pad=0):
    """torchvision BasicConv2d (conv, BN eps=1e-3 eval, ReLU)."""
    x = F.conv2d(x, sd[p + 'conv.weight'], None, stride, pad)
    x = F.batch_norm(x, sd[p + 'bn.running_mean'], sd[p + 'bn.running_var'], sd[p + 'bn.weight'],
                     sd[p + 'bn.bias'], False, 0.1, 1e-3)
    return F.relu(x)


def _incA(sd, p, x):
    b1 = _basic_conv(sd, p + 'branch1x1.', x)
    b5 = _basic_conv(sd, p + 'branch5x5_2.', _basic_conv(sd, p + 'branch5x5_1.', x), pad=2)
    b3 = _basic_conv(sd, p + 'branch3x3dbl_1.', x)
    b3 = _basic_conv(sd, p + 'branch3x3dbl_2.', b3, pad=1)
    b3 = _basic_conv(sd, p + 'branch3x3dbl_3.', b3, pad=1)
    bp = _basic_conv(sd, p + 'branch_pool.', F.avg_pool2d(x, 3, 1, 1))
    return torch.cat([b1, b5, b3, bp], 1)


def _incB(sd, p, x):
    b3 = _basic_conv(sd, p + 'branch3x3.', x, stride=2)
    bd = _basic_conv(sd, p + 'branch3x3dbl_1.', x)
    bd = _basic_conv(sd, p + 'branch3x3dbl_2.', bd, pad=1)
    bd = _basic_conv(sd, p + 'branch3x3dbl_3.', bd, stride=2)
    return torch.cat([b3, bd, F.max_pool2d(x, 3, 2)], 1)


def _incC(sd, p, x):
    b1 = _basic_conv(sd, p + 'branch1x1.', x)
    b7 = _basic_conv(sd, p + 'branch7x7_1.', x)
    b7 = _basic_conv(sd, p + 'branch7x7_2.', b7, pad=(0, 3))
    b7 = _basic_conv(sd, p + 'branch7x7_3.', b7, pad=(3, 0))
    bd = _basic_conv(sd, p + 'branch7x7dbl_1.', x)
    bd = _basic_conv(sd, p + 'branch7x7dbl_2.', bd, pad=(3, 0))
    bd = _basic_conv(sd, p + 'branch7x7dbl_3.', bd, pad=(0, 3))
    bd = _basic_conv(sd, p + 'branch7x7dbl_4.', bd, pad=(3, 0))
    bd = _basic_conv(sd, p + 'branch7x7dbl_5.', bd, pad=(0, 3))
    bp = _basic_conv(sd, p + 'branch_pool.', F.avg_pool2d(x, 3, 1, 1))
    return torch.cat([b1, b7, bd, bp], 1)


def _incD(sd, p, x):
    b3 = _basic_conv(sd, p + 'branch3x3_2.', _basic_conv(sd, p + 'branch3x3_1.', x), stride=2)
    b7 = _basic_conv(sd, p + 'branch7x7x3_1.', x)
    b7 = _basic_conv(sd, p + 'branch7x7x3_2.', b7, pad=(0, 3))
    b7 = _basic_conv(sd, p + 'branch7x7x3_3.', b7, pad=(3, 0))
    b7 = _basic_conv(sd, p + 'branch7x7x3_4.', b7, stride=2)
    return torch.cat([b3, b7, F.max_pool2d(x, 3, 2)], 1)


def _incE(sd, p, x):
    b1 = _basic_conv(sd, p + 'branch1x1.', x)
    b3 = _basic_conv(sd, p + 'branch3x3_1.', x)
    b3 = torch.cat([_basic_conv(sd, p + 'branch3x3_2a.', b3, pad=(0, 1)),
                    _basic_conv(sd, p + 'branch3x3_2b.', b3, pad=(1, 0))], 1)
    bd = _basic_conv(sd, p + 'branch3x3dbl_1.', x)
    bd = _basic_conv(sd, p + 'branch3x3dbl_2.', bd, pad=1)
    bd = torch.cat([_basic_conv(sd, p + 'branch3x3dbl_3a.', bd, pad=(0, 1)),
                    _basic_conv(sd, p + 'branch3x3dbl_3b.', bd, pad=(1, 0))], 1)
    bp = _basic_conv(sd, p + 'branch_pool.', F.avg_pool2d(x, 3, 1, 1))
    return torch.cat([b1, b3, bd, bp], 1)


def cnn_encoder(sd, x):
    """CNN_ENCODER.forward (DAMSM.py:170-230). PARITY UNPINNED: restated from
    torchvision's inception_v3 (absent here); frozen, eval-mode BN."""
    x = F.interpolate(x, size=(299, 299), mode='bilinear', align_corners=False)
    x = _basic_conv(sd, 'Conv2d_1a_3x3.', x, stride=2)
    x = _basic_conv(sd, 'Conv2d_2a_3x3.', x)
    x = _basic_conv(sd, 'Conv2d_2b_3x3.', x, pad=1)
    x = F.max_pool2d(x, 3, 2)
    x = _basic_conv(sd, 'Conv2d_3b_1x1.', x)
    x = _basic_conv(sd, 'Conv2d_4a_3x3.', x)
    x = F.max_pool2d(x, 3, 2)
    for n in ['Mixed_5b', 'Mixed_5c', 'Mixed_5d']:
        x = _incA(sd, n + '.', x)
    x = _incB(sd, 'Mixed_6a.', x)
    for n in ['Mixed_6b', 'Mixed_6c', 'Mixed_6d', 'Mixed_6e']:
        x = _incC(sd, n + '.', x)
    feats = x
    x = _incD(sd, 'Mixed_7a.', x)
    x = _incE(sd, 'Mixed_7b.', x)
    x = _incE(sd, 'Mixed_7c.', x)
    x = F.avg_pool2d(x, kernel_size=8).reshape(x.shape[0], -1)
    code = F.linear(x, sd['emb_cnn_code.weight'], sd['emb_cnn_code.bias'])
    feats = F.conv2d(feats, sd['emb_features.weight'])
    return feats, code


def fid_inception(sd, x, output_blocks=(3,)):
    """InceptionV3.forward of the FID leg (metrics/FID/inception.py:115-147).
    PARITY UNPINNED: the blocks are torchvision's inception_v3 (absent here),
    restated as in cnn_encoder; eval-mode BN.  x: (B, 3, H, W) in [0, 1]."""
    x = F.interpolate(x, size=(299, 299), mode='bilinear', align_corners=True)
    x = x.clone()
    x[:, 0] = x[:, 0] * (0.229 / 0.5) + (0.485 - 0.5) / 0.5
    x[:, 1] = x[:, 1] * (0.224 / 0.5) + (0.456 - 0.5) / 0.5
    x[:, 2] = x[:, 2] * (0.225 / 0.5) + (0.406 - 0.5) / 0.5
    out = []
    x = _basic_conv(sd, 'Conv2d_1a_3x3.', x, stride=2)
    x = _basic_conv(sd, 'Conv2d_2a_3x3.', x)
    x = F.max_pool2d(_basic_conv(sd, 'Conv2d_2b_3x3.', x, pad=1), 3, 2)
    if 0 in output_blocks:
        out.append(x)
    x = _basic_conv(sd, 'Conv2d_3b_1x1.', x)
    x = F.max_pool2d(_basic_conv(sd, 'Conv2d_4a_3x3.', x), 3, 2)
    if 1 in output_blocks:
        out.append(x)
    for n in ['Mixed_5b', 'Mixed_5c', 'Mixed_5d']:
        x = _incA(sd, n + '.', x)
    x = _incB(sd, 'Mixed_6a.', x)
    for n in ['Mixed_6b', 'Mixed_6c', 'Mixed_6d', 'Mixed_6e']:
        x = _incC(sd, n + '.', x)
    if 2 in output_blocks:
        out.append(x)
    x = _incE(sd, 'Mixed_7c.', _incE(sd, 'Mixed_7b.', _incD(sd, 'Mixed_7a.', x)))
    if 3 in output_blocks:
        out.append(F.adaptive_avg_pool2d(x, (1, 1)))
    return out


def standin_image_encoder(sd, x):
    """The small image encoder used by the golden full-step fixtures in place
    of Inception-v3 (which needs torchvision): regions = conv15x15/s15 (3->256)
    of the 256^2 image (17x17 grid); code = Linear(256,256)(mean of regions).
    Smaller images (the stage-1 slice's img_64) are first resized to 256^2
    (bilinear, align_corners=False -- as CNN_ENCODER resizes to 299,
    DAMSM.py:173)."""
    if x.shape[-1] != 256:
        x = F.interpolate(x, size=(256, 256), mode='bilinear', align_corners=False)
    regions = F.conv2d(x, sd['standin.regions.weight'], None, 15)
    code = F.linear(regions.mean(dim=(2, 3)), sd['standin.code.weight'], sd['standin.code.bias'])
    return regions, code


STANDIN_SPEC = [('standin.regions.weight', (256, 3, 15, 15)), ('standin.code.weight', (256, 256)),
                ('standin.code.bias', (256,))]
