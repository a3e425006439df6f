"""EE-GAN networks on MI355X (drop-in for the reference's models.py).

Same class names, constructor arguments, forward signatures and state_dict
keys as models.py:14-403; every layer runs on libeegan_hip.so:

* convs are implicit-GEMM bf16 MFMA kernels over NHWC activations with the
  following activation fused into the epilogue;
* SyncBN + affine_ssa modulation + ReLU (+ the nearest-2x upsample of
  Gen.SAGB_progress) is one fused apply kernel after a statistics kernel;
* the learnable 1x1 shortcut of an upsampling SAGB block runs at the LOW
  resolution before the upsample (nearest-up commutes with a 1x1 conv), and
  resD's 1x1 shortcut runs AFTER the 2x2 average pool (they commute too):
  identical math, 4x fewer FLOPs than models.py:108-111 / 280-285.

Activations are bf16 NHWC tensors with the reference's logical NCHW shape;
fp32 NCHW inputs (e.g. real images from the reference data pipeline) are
accepted and converted.
"""
from collections import OrderedDict
import math

import torch
import torch.nn as nn

from miscc.config import cfg
from sync_batchnorm import SynchronizedBatchNorm2d
from eegan_hip import functional as Fn
from eegan_hip import dist as D
from eegan_hip.nn import Conv2d, Linear

BatchNorm = SynchronizedBatchNorm2d


def conv1x1(in_channel, out_channel):
    return Conv2d(in_channel, out_channel, kernel_size=1, stride=1, padding=0, bias=False)


def conv3x3(in_channel, out_channel):
    return Conv2d(in_channel, out_channel, kernel_size=3, stride=1, padding=1, bias=False)


def conv4x4(in_channel, out_channel):
    return Conv2d(in_channel, out_channel, kernel_size=4, stride=2, padding=1, bias=False)


class _ImageHead(nn.Sequential):
    """get_image (models.py:25-32): BN -> LeakyReLU(0.2) -> conv3x3 -> tanh.
    Keys: 0.{weight,bias,running_*}, 2.weight."""

    def forward(self, x):
        h = self[0](x, act='lrelu', slope=0.2)
        return self[2](h, act='tanh')


def get_image(in_channel, out_channel=3):
    return _ImageHead(BatchNorm(in_channel), nn.LeakyReLU(0.2, inplace=True),
                      Conv2d(in_channel, out_channel, kernel_size=3, padding=1, bias=False), nn.Tanh())


class _MaskHead(nn.Sequential):
    """get_mask (models.py:34-41): conv3x3 -> BN(100) -> ReLU -> conv1x1 -> fp32 (N,1,H,W)."""

    def forward(self, x):
        h = self[0](x)
        h = self[1](h, act='relu')
        return self[3](h, out_f32=True)


def get_mask(in_channel, mask_channel=100, out_channel=1):
    return _MaskHead(conv3x3(in_channel, mask_channel), BatchNorm(mask_channel), nn.ReLU(),
                     conv1x1(mask_channel, out_channel))


class _MLP(nn.Sequential):
    def forward(self, x):
        return self.linear2(self.linear1(x, act='relu'))


class affine_ssa(nn.Module):
    """models.py:43-86: (gamma(c)*m + 1) * BN_noaffine(x) + beta(c)*m."""

    def __init__(self, num_features, ntf=cfg.TEXT.EMBEDDING_DIM, norm_layer=BatchNorm):
        super().__init__()
        self.norm2d = norm_layer(num_features, affine=False)
        self.fc_gamma = _MLP(OrderedDict([('linear1', Linear(ntf, 256)), ('relu1', nn.ReLU(inplace=True)),
                                          ('linear2', Linear(256, num_features))]))
        self.fc_beta = _MLP(OrderedDict([('linear1', Linear(ntf, 256)), ('relu1', nn.ReLU(inplace=True)),
                                         ('linear2', Linear(256, num_features))]))
        self._initialize()

    def _initialize(self):
        for m in (self.fc_gamma.linear2, self.fc_beta.linear2):
            nn.init.zeros_(m.weight.data)
            nn.init.zeros_(m.bias.data)

    def mlp_params(self):
        """(W1, b1, W2, b2) of fc_gamma then fc_beta (Fn.AffineMLPsFn order)."""
        out = []
        for m in (self.fc_gamma, self.fc_beta):
            out += [m.linear1.weight, m.linear1.bias, m.linear2.weight, m.linear2.bias]
        return out

    def forward(self, feat, cond, semi_mask, act=None, up2=False, gb=None):
        """`gb` = precomputed (gamma, beta) MLP outputs (Gen batches all of them)."""
        if gb is not None:
            gam, bet = gb
        else:
            gam = self.fc_gamma(cond)
            bet = self.fc_beta(cond)
        if gam.dim() == 1:
            gam = gam.unsqueeze(0)
        if bet.dim() == 1:
            bet = bet.unsqueeze(0)
        return self.norm2d.modulate(feat, gam, bet, semi_mask, act=act, up2=up2)


class SAGB_Block(nn.Module):
    """Spatial affine generative block (models.py:89-126)."""

    def __init__(self, in_ch, out_ch, affine_blocks=None, pred_mask=True):
        super().__init__()
        if affine_blocks is None:
            affine_blocks = [affine_ssa, affine_ssa]
        self.learnable_sc = in_ch != out_ch
        self.pred_mask = pred_mask
        self.c1 = conv3x3(in_ch, out_ch)
        self.c2 = conv3x3(out_ch, out_ch)
        self.affine1 = affine_blocks[0](in_ch)
        self.affine2 = affine_blocks[1](out_ch)
        self.gamma = nn.Parameter(torch.zeros(1))
        if self.learnable_sc:
            self.c_sc = Conv2d(in_ch, out_ch, 1, stride=1, padding=0)
        if self.pred_mask:
            self.conv_mask = get_mask(out_ch)

    def shortcut(self, x, up2=False):
        if self.learnable_sc:
            x = self.c_sc(x)          # at low resolution when up2 (commutes with nearest-up)
        return Fn.Upsample2Fn.apply(x) if up2 else x

    def residual(self, feat, conds, semi_mask, up2=False, gb=None):
        gb = gb or (None, None)
        h = self.affine1(feat, conds[0], semi_mask, act='relu', up2=up2, gb=gb[0])
        h = self.c1(h)
        h = self.affine2(h, conds[1], semi_mask, act='relu', gb=gb[1])
        return self.c2(h)

    def forward(self, feat, conds, semi_mask, up2=False, gb=None):
        """`up2=True` consumes the PRE-upsample feature map (fusing the
        F.interpolate(scale_factor=2) of Gen.SAGB_progress, models.py:219).
        `gb` = ((gamma1, beta1), (gamma2, beta2)) precomputed by Gen."""
        c_feat = Fn.ScaleAddFn.apply(self.shortcut(feat, up2), self.residual(feat, conds, semi_mask, up2, gb),
                                     self.gamma)
        c_semi_mask = self.conv_mask(c_feat) if self.pred_mask else None
        return c_feat, c_semi_mask


class Cum_Block(nn.Module):
    """models.py:129-143: fuse(conv3x3(up2(conv1x1(prev))) + gamma * cur)."""

    def __init__(self, prev_channel, cur_channel):
        super().__init__()
        self.up_block = nn.Sequential(conv1x1(prev_channel, cur_channel), nn.Upsample(scale_factor=2, mode='nearest'),
                                      conv3x3(cur_channel, cur_channel))
        self.fuse_block = conv3x3(cur_channel, cur_channel)
        self.gamma = nn.Parameter(torch.zeros(1))

    def up(self, prev_feat):
        u = self.up_block[0](prev_feat)
        return self.up_block[2](u, up2=True)  # nearest-2x folded into the conv's input gather

    def fuse(self, u, cur_feat):
        return self.fuse_block(Fn.ScaleAddFn.apply(u, cur_feat, self.gamma))

    def forward(self, prev_feat, cur_feat):
        return self.fuse(self.up(prev_feat), cur_feat)


class ATTR_Enhance(nn.Module):
    """models.py:146-180 (softmax(QK^T) * 1/sqrt(ntf), then V)."""

    def __init__(self, ntf=cfg.TEXT.EMBEDDING_DIM):
        super().__init__()
        D.guard_state_dict(self)   # a rank whose collectives failed must not checkpoint
        self.attr_query = Linear(ntf, ntf)
        self.attr_key = Linear(ntf, ntf)
        self.attr_value = Linear(ntf, ntf)
        self._norm_fact = 1 / math.sqrt(ntf)

    def forward(self, sent, attrs):
        D.ensure_grad_hooks(self)   # data-parallel gradient averaging (no-op at world 1)
        combine = torch.cat([sent.unsqueeze(1), attrs], dim=1).float()
        q = self.attr_query(combine)
        k = self.attr_key(combine)
        v = self.attr_value(combine)
        attn_attrs = Fn.AttrAttnFn.apply(q, k, v, self._norm_fact)
        return attn_attrs[:, 0, :], attn_attrs

    @staticmethod
    def attr_merge(attn_attrs):
        return attn_attrs.sum(dim=1)


# Gen.forward_branched: cum_64's upsampling branch beside SAGB block 4 (False: after it;
# in-process A/B -0.4 %, profiles/r04_gen_side_u64_ab.txt)
GEN_SIDE_U64 = False


class Gen(nn.Module):
    """models.py:183-256."""

    def __init__(self, ngf=cfg.GAN.GF_DIM, nz=cfg.GAN.Z_DIM):
        super().__init__()
        D.guard_state_dict(self)   # a rank whose collectives failed must not checkpoint
        self.ngf = ngf
        self.fc = Linear(nz, ngf * 8 * 4 * 4)
        self.blocks = nn.ModuleList([
            SAGB_Block(ngf * 8, ngf * 8, [affine_ssa, affine_ssa], pred_mask=True),
            SAGB_Block(ngf * 8, ngf * 8, [affine_ssa, affine_ssa], pred_mask=True),
            SAGB_Block(ngf * 8, ngf * 8, [affine_ssa, affine_ssa], pred_mask=True),
            SAGB_Block(ngf * 8, ngf * 8, [affine_ssa, affine_ssa], pred_mask=True),
            SAGB_Block(ngf * 8, ngf * 4, [affine_ssa, affine_ssa], pred_mask=True),
            SAGB_Block(ngf * 4, ngf * 2, [affine_ssa, affine_ssa], pred_mask=True),
            SAGB_Block(ngf * 2, ngf * 1, [affine_ssa, affine_ssa], pred_mask=False),
        ])
        self.cum_64 = Cum_Block(ngf * 8, ngf * 4)
        self.cum_128 = Cum_Block(ngf * 4, ngf * 2)
        self.cum_256 = Cum_Block(ngf * 2, ngf * 1)
        self.get_image_64 = get_image(ngf * 4, 3)
        self.get_image_128 = get_image(ngf * 2, 3)
        self.get_image_256 = get_image(ngf, 3)
        self.init_mask = get_mask(ngf * 8)
        self.scales = [4, 8, 16, 32, 64, 128, 256]
        self.stages = 3  # 1: the harness stage-1 slice (img_64 only)
        # a HIP stream the trainer lends (None: one stream): the Cum_Block / image
        # branches of stages 2-3 run on it beside SAGB blocks 5-6 (forward_branched)
        self.side_stream = None

    @staticmethod
    def SAGB_progress(feat, conds, stage_mask, scale, SAGB_block, gb=None):
        fusion_mask = Fn.MaskResizeSigmoidFn.apply(stage_mask, scale)
        return SAGB_block(feat, conds, fusion_mask, up2=True, gb=gb)

    def affine_mlps(self, sent, attrs):
        """gamma/beta of every affine_ssa the pass uses, in grouped launches
        (Fn.AffineMLPsFn); blocks 0-3 condition both affines on sent, blocks
        4-6 affine1 on sent and affine2 on attrs (models.py:214-236)."""
        nblk = 5 if self.stages == 1 else 7
        order = [(b, 0) for b in range(nblk)] + [(b, 1) for b in range(4)] + [(b, 1) for b in range(4, nblk)]
        cidx, params = [], []
        for b, k in order:
            aff = self.blocks[b].affine1 if k == 0 else self.blocks[b].affine2
            c = 1 if (k == 1 and b >= 4) else 0
            cidx += [c, c]
            params += aff.mlp_params()
        outs = Fn.AffineMLPsFn.apply(sent, attrs, *params, tuple(cidx), 2)
        gb = [[None, None] for _ in range(nblk)]
        for i, (b, k) in enumerate(order):
            gb[b][k] = (outs[2 * i], outs[2 * i + 1])
        return gb

    def forward(self, x, sent, attrs):
        D.ensure_grad_hooks(self)
        gb = self.affine_mlps(sent, attrs) if Fn.GROUPED_MLP else [None] * 7
        out = self.fc(x.float())
        out = Fn.FcToNhwcFn.apply(out, 8 * self.ngf)
        stage_mask = self.init_mask(out)
        fusion_mask = Fn.MaskResizeSigmoidFn.apply(stage_mask, 4)
        out, stage_mask = self.blocks[0](out, [sent, sent], fusion_mask, gb=gb[0])
        for ix, scale in enumerate([8, 16, 32]):
            out, stage_mask = self.SAGB_progress(out, [sent, sent], stage_mask, scale, self.blocks[ix + 1],
                                                 gb[ix + 1])
        x_32 = out
        if self.stages == 3 and self.side_stream is not None:
            return self.forward_branched(x_32, stage_mask, sent, attrs, gb)
        # the same operations as models.py:244-256, created in forward_branched's
        # order: autograd runs backward nodes by creation order, so the gradients of
        # multi-consumer activations (x_64, x_128, the masks) are summed in the same
        # order on one stream and on two -- bit-identical parameter gradients
        x_64, stage_mask = self.SAGB_progress(x_32, [sent, attrs], stage_mask, 64, self.blocks[4], gb[4])
        cum_x_64 = self.cum_64(x_32, x_64)
        img_64 = self.get_image_64(cum_x_64)
        if self.stages == 1:
            return [img_64]
        u_128 = self.cum_128.up(cum_x_64)
        x_128, stage_mask = self.SAGB_progress(x_64, [sent, attrs], stage_mask, 128, self.blocks[5], gb[5])
        cum_x_128 = self.cum_128.fuse(u_128, x_128)
        img_128 = self.get_image_128(cum_x_128)
        u_256 = self.cum_256.up(cum_x_128)
        x_256, _ = self.SAGB_progress(x_128, [sent, attrs], stage_mask, 256, self.blocks[6], gb[6])
        cum_x_256 = self.cum_256.fuse(u_256, x_256)
        img_256 = self.get_image_256(cum_x_256)
        return [img_64, img_128, img_256]

    def forward_branched(self, x_32, stage_mask, sent, attrs, gb):
        """Stages 1 (from block 4) to 3 as two streams: SAGB blocks 4-6 (the
        x_64 / x_128 / x_256 chain, with the masks) on the caller's stream; the
        Cum_Blocks, the image heads and each Cum_Block's upsampling branch on
        `side_stream`, which depends only on x_32 / x_64 / x_128.  The same
        operations on the same inputs as forward(); their backward nodes run on
        the stream of their forward (autograd), so the generator's backward
        splits the same way."""
        main, side = torch.cuda.current_stream(), self.side_stream
        # Every tensor crossing between the streams is (1) recorded on its reader, since
        # it is saved for backward and the last reference may drop on the other stream,
        # and (2) read through Fn.StreamHandoffFn, whose backward records the gradient
        # flowing back across on the stream that consumes it: the caching allocator
        # must not hand either memory to the producing stream's next allocation
        # before the other stream's queued reads ran.
        hand = Fn.StreamHandoffFn.apply
        x_32.record_stream(side)
        u_64 = None
        if GEN_SIDE_U64:
            side.wait_stream(main)
            with torch.cuda.stream(side):
                u_64 = self.cum_64.up(hand(x_32, main))
        x_64, stage_mask = self.SAGB_progress(x_32, [sent, attrs], stage_mask, 64, self.blocks[4], gb[4])
        x_64.record_stream(side)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            cum_x_64 = self.cum_64.fuse(u_64 if u_64 is not None else self.cum_64.up(hand(x_32, main)),
                                        hand(x_64, main))
            img_64 = self.get_image_64(cum_x_64)
            u_128 = self.cum_128.up(cum_x_64)
        x_128, stage_mask = self.SAGB_progress(x_64, [sent, attrs], stage_mask, 128, self.blocks[5], gb[5])
        x_128.record_stream(side)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            cum_x_128 = self.cum_128.fuse(u_128, hand(x_128, main))
            img_128 = self.get_image_128(cum_x_128)
            u_256 = self.cum_256.up(cum_x_128)
        x_256, _ = self.SAGB_progress(x_128, [sent, attrs], stage_mask, 256, self.blocks[6], gb[6])
        main.wait_stream(side)
        u_256.record_stream(main)
        cum_x_256 = self.cum_256.fuse(hand(u_256, side), x_256)
        img_256 = self.get_image_256(cum_x_256)
        return [img_64, img_128, img_256]


# ---------------------------------------------------------------- discriminators
class resD(nn.Module):
    """models.py:262-288: avg_pool(conv_s(x)) + gamma * lrelu(conv3x3(lrelu(conv4x4s2(x))))."""

    def __init__(self, fin, fout, downsample=True):
        super().__init__()
        self.downsample = downsample
        self.learned_shortcut = (fin != fout)
        self.conv_r = nn.Sequential(Conv2d(fin, fout, 4, 2, 1, bias=False), nn.LeakyReLU(0.2, inplace=True),
                                    Conv2d(fout, fout, 3, 1, 1, bias=False), nn.LeakyReLU(0.2, inplace=True))
        self.conv_s = Conv2d(fin, fout, 1, stride=1, padding=0)
        self.gamma = nn.Parameter(torch.zeros(1))

    def forward(self, x):
        # residual()'s last LeakyReLU is deferred to ScaleAddFn's backward (first-order
        # only: under create_graph ScaleAddFn does not gate, so conv_r[2] keeps its ActBwdFn)
        lrelu = Fn.ACT_CODES['lrelu']
        if self.downsample and Fn.FUSE_ACT_BWD:
            # the shortcut's pooling and conv_r[0] read x together (Fn.PoolConvFn: one dx)
            c0 = self.conv_r[0]
            xp, h = Fn.PoolConvFn.apply(x, c0.weight, c0.bias, c0.geom(False), lrelu, 0.2, c0._cache, True)
            sc = self.conv_s(xp) if self.learned_shortcut else xp
            r = self.conv_r[2](h, act='lrelu', slope=0.2, in_act='lrelu', defer_act='first_order')
            return Fn.ScaleAddFn.apply(sc, r, self.gamma, lrelu, 0.2)
        return Fn.ScaleAddFn.apply(self.shortcut(x), self.residual(x), self.gamma, lrelu, 0.2)

    def shortcut(self, x):
        if self.downsample:
            x = Fn.AvgPool2Fn.apply(x)      # pool first: commutes with the 1x1 conv (+bias)
        if self.learned_shortcut:
            x = self.conv_s(x)
        return x

    def residual(self, x):
        # each LeakyReLU's backward runs inside its only consumer's backward
        # (the next conv's data gradient, ScaleAddFn): Conv2dFn in_act / defer_act
        h = self.conv_r[0](x, act='lrelu', slope=0.2, defer_act=True)
        return self.conv_r[2](h, act='lrelu', slope=0.2, in_act='lrelu', defer_act='first_order')


class DiscSent(nn.Module):
    """models.py:290-306 -> fp32 (N,1,1,1)."""

    def __init__(self, ndf, nef):
        super().__init__()
        self.df_dim = ndf
        self.ef_dim = nef
        self.joint_conv = nn.Sequential(Conv2d(ndf + nef, ndf * 2, 3, 1, 1, bias=False),
                                        nn.LeakyReLU(0.2, inplace=True), Conv2d(ndf * 2, 1, 4, 1, 0, bias=False))

    def forward(self, feat, cond):
        h = Fn.CatTileFn.apply(feat, cond.reshape(-1, self.ef_dim))
        h = self.joint_conv[0](h, act='lrelu', slope=0.2, defer_act=True)
        return self.joint_conv[2](h, out_f32=True, in_act='lrelu')


class DiscCond(nn.Module):
    """models.py:308-338 -> (pair (N,), class logits (N, class_nums)), fp32."""

    def __init__(self, ndf, nef, class_nums=200):
        super().__init__()
        self.ndf = ndf
        self.nef = nef
        self.class_nums = class_nums
        self.joinConv = nn.Sequential(Conv2d(ndf + nef, ndf * 2, 3, 1, 1, bias=False), nn.LeakyReLU(0.2, inplace=True))
        self.pair_node = Conv2d(ndf * 2, 1, kernel_size=4, stride=4)
        self.class_node = Conv2d(ndf * 2, ndf * 2, kernel_size=4, stride=4)
        self.class_linear = Linear(ndf * 2, self.class_nums)

    def forward(self, img_code, c_code):
        h = Fn.CatTileFn.apply(img_code, c_code.reshape(-1, self.nef))
        h = self.joinConv[0](h, act='lrelu', slope=0.2, defer_act=True)  # both consumers gate
        pair = self.pair_node(h, out_f32=True, in_act='lrelu').reshape(-1)
        cls = self.class_node(h, out_f32=True, in_act='lrelu').reshape(-1, self.ndf * 2)
        return pair, self.class_linear(cls)


class _DisBase(nn.Module):
    def __init__(self):
        super().__init__()
        D.guard_state_dict(self)   # a rank whose collectives failed must not checkpoint

    def _stem(self, x):
        D.ensure_grad_hooks(self)   # covers COND_DNET, which train.py calls outside forward
        if x.dtype != torch.bfloat16:
            x = Fn.ImageToNhwcFn.apply(x)
        return self.conv_img(x)


class Dis64(_DisBase):
    def __init__(self, ndf=cfg.GAN.DF_DIM):
        super().__init__()
        self.conv_img = Conv2d(3, ndf, 3, 1, 1)
        self.block0 = resD(ndf * 1, ndf * 2)
        self.block1 = resD(ndf * 2, ndf * 4)
        self.block2 = resD(ndf * 4, ndf * 8)
        self.block3 = resD(ndf * 8, ndf * 8)
        self.COND_DNET = DiscSent(ndf * 8, 256)

    def forward(self, x):
        out = self._stem(x)
        for b in (self.block0, self.block1, self.block2, self.block3):
            out = b(out)
        return out


class Dis128(_DisBase):
    def __init__(self, ndf=cfg.GAN.DF_DIM):
        super().__init__()
        self.conv_img = Conv2d(3, ndf, 3, 1, 1)
        self.block0 = resD(ndf * 1, ndf * 2)
        self.block1 = resD(ndf * 2, ndf * 4)
        self.block2 = resD(ndf * 4, ndf * 8)
        self.block3 = resD(ndf * 8, ndf * 8)
        self.block4 = resD(ndf * 8, ndf * 16)
        self.COND_DNET = DiscSent(ndf * 16, 256)

    def forward(self, x):
        out = self._stem(x)
        for b in (self.block0, self.block1, self.block2, self.block3, self.block4):
            out = b(out)
        return out


class Dis256(_DisBase):
    def __init__(self, ndf, disc_class, class_nums):
        super().__init__()
        self.conv_img = Conv2d(3, ndf, 3, 1, 1)
        self.block0 = resD(ndf * 1, ndf * 2)
        self.block1 = resD(ndf * 2, ndf * 4)
        self.block2 = resD(ndf * 4, ndf * 8)
        self.block3 = resD(ndf * 8, ndf * 16)
        self.block4 = resD(ndf * 16, ndf * 16)
        self.block5 = resD(ndf * 16, ndf * 16)
        self.disc_class = disc_class
        if disc_class:
            self.COND_DNET = DiscCond(ndf * 16, 256, class_nums=class_nums)
        else:
            self.COND_DNET = DiscSent(ndf * 16, 256)

    def forward(self, x):
        out = self._stem(x)
        for b in (self.block0, self.block1, self.block2, self.block3, self.block4, self.block5):
            out = b(out)
        return out
