"""Frozen DAMSM encoders (API of DAMSM.py:30-230).

RNN_ENCODER: embedding + bidirectional LSTM (eval mode) as HIP kernels --
one fp32 GEMM per direction for the input projections and one recurrence
kernel with lengths read on the device (no pack_padded_sequence).

CNN_ENCODER: Inception-v3 up to Mixed_7c with torchvision's module / key
names (the pretrained AttnGAN image_encoder200.pth loads unchanged), defined
here because torchvision is not a dependency.  Frozen and in eval mode in the
training step (train.py:241-248), so every BasicConv2d's BatchNorm is folded
into the conv weights/bias and the ReLU into the conv epilogue; the encoder
runs forward + input-gradient backward on the bf16 MFMA conv kernels.
"""
import os

import torch
import torch.nn as nn

from miscc.config import cfg
from eegan_hip import functional as Fn
from eegan_hip.nn import Conv2d, Linear
from eegan_hip._lib import ops
from eegan_hip.tensor import stream, F32


def conv1x1(in_planes, out_planes, bias=False):
    return Conv2d(in_planes, out_planes, kernel_size=1, stride=1, padding=0, bias=bias)


class RNN_ENCODER(nn.Module):
    def __init__(self, ntoken, ninput=300, drop_prob=0.5, nhidden=128, nlayers=1, bidirectional=True):
        super().__init__()
        self.n_steps = cfg.TEXT.WORDS_NUM
        self.ntoken = ntoken
        self.ninput = ninput
        self.drop_prob = drop_prob
        self.nlayers = nlayers
        self.bidirectional = bidirectional
        self.rnn_type = cfg.RNN_TYPE
        self.num_directions = 2 if bidirectional else 1
        self.nhidden = nhidden // self.num_directions
        if self.rnn_type != 'LSTM' or nlayers != 1 or not bidirectional:
            raise NotImplementedError('the DAMSM text encoder is a 1-layer bidirectional LSTM')
        self.encoder = nn.Embedding(ntoken, ninput)
        self.drop = nn.Dropout(drop_prob)
        self.rnn = nn.LSTM(ninput, self.nhidden, nlayers, batch_first=True, dropout=0.0, bidirectional=True)
        self.encoder.weight.data.uniform_(-0.1, 0.1)
        self._cache_key = None

    def init_hidden(self, bsz):
        w = next(self.parameters()).data
        z = w.new_zeros(self.nlayers * self.num_directions, bsz, self.nhidden)
        return (z, z.clone())

    def _weights(self):
        r = self.rnn
        key = tuple((p.data_ptr(), p._version) for p in r.parameters())
        if key != self._cache_key:
            H = self.nhidden
            self._wih = [r.weight_ih_l0.detach().float().contiguous(), r.weight_ih_l0_reverse.detach().float().contiguous()]
            self._bias = [(r.bias_ih_l0 + r.bias_hh_l0).detach().float().contiguous(),
                          (r.bias_ih_l0_reverse + r.bias_hh_l0_reverse).detach().float().contiguous()]
            self._whhT = torch.stack([r.weight_hh_l0.detach().t(), r.weight_hh_l0_reverse.detach().t()]).float().contiguous()
            self._cache_key = key
        return self._wih, self._bias, self._whhT

    def forward(self, captions, cap_lens, hidden=None, mask=None, max_len=None):
        """(B, T) int64 tokens -> words (B, 2H, T_max) fp32, sent (B, 2H) fp32.
        T_max = max(cap_lens) as pad_packed_sequence produces; pass `max_len`
        to avoid reading the lengths on the host."""
        dev = self.encoder.weight.device
        caps = captions.to(dev).long().contiguous()
        if caps.dim() == 1:
            caps = caps.unsqueeze(0)
        B, T = caps.shape
        lens = torch.as_tensor(cap_lens).to(device=dev, dtype=torch.long).reshape(-1).contiguous()
        Tout = int(max_len) if max_len is not None else int(lens.max().item())
        E, H = self.ninput, self.nhidden
        s = stream()
        emb = torch.empty((B * T, E), dtype=F32, device=dev)
        ops.embedding(caps.data_ptr(), B * T, self.encoder.weight.data_ptr(), E, emb.data_ptr(), s)
        if self.training and self.drop_prob > 0:
            emb = self.drop(emb)
        wih, bias, whhT = self._weights()
        xproj = torch.empty((2, B * T, 4 * H), dtype=F32, device=dev)
        for d in range(2):
            ops.gemm_f32(emb.data_ptr(), E, 1, wih[d].data_ptr(), 1, E, xproj[d].data_ptr(), 4 * H, B * T, 4 * H, E,
                         bias[d].data_ptr(), 0, 1.0, 0.0, s)
        words = torch.empty((B, 2 * H, Tout), dtype=F32, device=dev)
        sent = torch.empty((B, 2 * H), dtype=F32, device=dev)
        ops.lstm_bidir(xproj.data_ptr(), whhT.data_ptr(), lens.data_ptr(), B, T, H, Tout, words.data_ptr(),
                       sent.data_ptr(), s)
        return words, sent


# ------------------------------------------------------------- Inception-v3
class BatchNorm2dFrozen(nn.Module):
    """Parameter/buffer holder with nn.BatchNorm2d's names (eps 1e-3 as torchvision)."""

    def __init__(self, C, eps=0.001):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(C))
        self.bias = nn.Parameter(torch.zeros(C))
        self.register_buffer('running_mean', torch.zeros(C))
        self.register_buffer('running_var', torch.ones(C))
        self.register_buffer('num_batches_tracked', torch.tensor(0, dtype=torch.long))


class BasicConv2d(nn.Module):
    """conv (no bias) -> BN(eps=1e-3, running stats) -> ReLU, BN folded into the packed weights."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0):
        super().__init__()
        self.conv = Conv2d(in_channels, out_channels, kernel_size, stride=stride, padding=padding, bias=False)
        self.bn = BatchNorm2dFrozen(out_channels)
        self._fold_key = None

    def _fold(self):
        bn = self.bn
        key = (bn.weight._version, bn.bias._version, bn.running_mean._version, bn.running_var._version,
               self.conv.weight._version, bn.weight.data_ptr())
        if key != self._fold_key:
            with torch.no_grad():
                scale = (bn.weight / torch.sqrt(bn.running_var + bn.eps)).float().contiguous()
                self._shift = (bn.bias - bn.running_mean * scale).float().contiguous()
            self._cache = Fn.PackCache(scale)
            self._fold_key = key
        return self._shift

    def forward(self, x, in_relu=False, defer=False):
        """in_relu: x is the ReLU output of a BasicConv2d called with defer=True
        whose consumers all gate (branch chains below): that ReLU's backward
        runs in this conv's data-gradient epilogue (Fn.Conv2dFn in_act/defer_act)."""
        shift = self._fold()
        return Fn.Conv2dFn.apply(x, self.conv.weight, shift, self.conv.geom(False), 1, 0.0, False, self._cache,
                                 1 if in_relu else 0, 0.0, defer)


def _chain(x, convs):
    """x -> convs[0] -> ... -> convs[-1]; every inner ReLU has one consumer, so
    its backward is fused into the next conv's data gradient."""
    for i, m in enumerate(convs):
        x = m(x, in_relu=i > 0, defer=i + 1 < len(convs))
    return x


def _cat(parts):
    return Fn.CatChannelsFn.apply(*parts)


# EEGAN_FUSE_1X1=0: the branch 1x1 convs that share a block input run separately.
FUSE_1X1 = os.environ.get('EEGAN_FUSE_1X1', '1') != '0'


class _Stacked1x1:
    """The 1x1 BasicConv2d branches of an Inception block that read the same
    input, run as ONE conv with their (BN-folded) weights stacked along the
    output channels; the branches take channel-slice views of its output
    (Fn.SplitChannelsFn).  Forward: 1 launch instead of k; backward: one data
    gradient over the assembled slice gradients instead of k of them and k-1
    gradient adds.  Frozen encoder: the stacked weights are rebuilt only when
    a member's parameters or BN statistics change."""

    def __init__(self, mods):
        self.mods = list(mods)
        self.key = None

    def _build(self):
        key = tuple((m.bn.weight._version, m.bn.bias._version, m.bn.running_mean._version,
                     m.bn.running_var._version, m.conv.weight._version, m.conv.weight.data_ptr()) for m in self.mods)
        if key != self.key:
            with torch.no_grad():
                ws, scales, shifts = [], [], []
                for m in self.mods:
                    bn = m.bn
                    sc = (bn.weight / torch.sqrt(bn.running_var + bn.eps)).float()
                    ws.append(m.conv.weight.detach().float())
                    scales.append(sc)
                    shifts.append((bn.bias - bn.running_mean * sc).float())
                self.W = torch.cat(ws, 0).contiguous(memory_format=torch.channels_last)
                self.shift = torch.cat(shifts).contiguous()
                self.cache = Fn.PackCache(torch.cat(scales).contiguous())
                self.sizes = tuple(m.conv.out_channels for m in self.mods)
                self.geom = Fn.Geom(sum(self.sizes), 1, 1, 1, 0, 0, 0)
            self.key = key

    def __call__(self, x):
        if not FUSE_1X1:
            return tuple(m(x) for m in self.mods)
        self._build()
        y = Fn.Conv2dFn.apply(x, self.W, self.shift, self.geom, 1, 0.0, False, self.cache)
        return Fn.SplitChannelsFn.apply(y, self.sizes)


class InceptionA(nn.Module):
    def __init__(self, in_channels, pool_features):
        super().__init__()
        self.branch1x1 = BasicConv2d(in_channels, 64, 1)
        self.branch5x5_1 = BasicConv2d(in_channels, 48, 1)
        self.branch5x5_2 = BasicConv2d(48, 64, 5, padding=2)
        self.branch3x3dbl_1 = BasicConv2d(in_channels, 64, 1)
        self.branch3x3dbl_2 = BasicConv2d(64, 96, 3, padding=1)
        self.branch3x3dbl_3 = BasicConv2d(96, 96, 3, padding=1)
        self.branch_pool = BasicConv2d(in_channels, pool_features, 1)
        self._stem = _Stacked1x1([self.branch1x1, self.branch5x5_1, self.branch3x3dbl_1])

    def forward(self, x):
        b1, t5, t3 = self._stem(x)
        b5 = _chain(t5, (self.branch5x5_2,))
        b3 = _chain(t3, (self.branch3x3dbl_2, self.branch3x3dbl_3))
        bp = self.branch_pool(Fn.AvgPool3s1Fn.apply(x))
        return _cat([b1, b5, b3, bp])


class InceptionB(nn.Module):
    def __init__(self, in_channels):
        super().__init__()
        self.branch3x3 = BasicConv2d(in_channels, 384, 3, stride=2)
        self.branch3x3dbl_1 = BasicConv2d(in_channels, 64, 1)
        self.branch3x3dbl_2 = BasicConv2d(64, 96, 3, padding=1)
        self.branch3x3dbl_3 = BasicConv2d(96, 96, 3, stride=2)

    def forward(self, x):
        b3 = self.branch3x3(x)
        bd = _chain(x, (self.branch3x3dbl_1, self.branch3x3dbl_2, self.branch3x3dbl_3))
        return _cat([b3, bd, Fn.MaxPool3s2Fn.apply(x)])


class InceptionC(nn.Module):
    def __init__(self, in_channels, channels_7x7):
        super().__init__()
        c7 = channels_7x7
        self.branch1x1 = BasicConv2d(in_channels, 192, 1)
        self.branch7x7_1 = BasicConv2d(in_channels, c7, 1)
        self.branch7x7_2 = BasicConv2d(c7, c7, (1, 7), padding=(0, 3))
        self.branch7x7_3 = BasicConv2d(c7, 192, (7, 1), padding=(3, 0))
        self.branch7x7dbl_1 = BasicConv2d(in_channels, c7, 1)
        self.branch7x7dbl_2 = BasicConv2d(c7, c7, (7, 1), padding=(3, 0))
        self.branch7x7dbl_3 = BasicConv2d(c7, c7, (1, 7), padding=(0, 3))
        self.branch7x7dbl_4 = BasicConv2d(c7, c7, (7, 1), padding=(3, 0))
        self.branch7x7dbl_5 = BasicConv2d(c7, 192, (1, 7), padding=(0, 3))
        self.branch_pool = BasicConv2d(in_channels, 192, 1)
        self._stem = _Stacked1x1([self.branch1x1, self.branch7x7_1, self.branch7x7dbl_1])

    def forward(self, x):
        b1, t7, td = self._stem(x)
        b7 = _chain(t7, (self.branch7x7_2, self.branch7x7_3))
        bd = _chain(td, (self.branch7x7dbl_2, self.branch7x7dbl_3, self.branch7x7dbl_4, self.branch7x7dbl_5))
        bp = self.branch_pool(Fn.AvgPool3s1Fn.apply(x))
        return _cat([b1, b7, bd, bp])


class InceptionD(nn.Module):
    def __init__(self, in_channels):
        super().__init__()
        self.branch3x3_1 = BasicConv2d(in_channels, 192, 1)
        self.branch3x3_2 = BasicConv2d(192, 320, 3, stride=2)
        self.branch7x7x3_1 = BasicConv2d(in_channels, 192, 1)
        self.branch7x7x3_2 = BasicConv2d(192, 192, (1, 7), padding=(0, 3))
        self.branch7x7x3_3 = BasicConv2d(192, 192, (7, 1), padding=(3, 0))
        self.branch7x7x3_4 = BasicConv2d(192, 192, 3, stride=2)
        self._stem = _Stacked1x1([self.branch3x3_1, self.branch7x7x3_1])

    def forward(self, x):
        t3, t7 = self._stem(x)
        b3 = _chain(t3, (self.branch3x3_2,))
        b7 = _chain(t7, (self.branch7x7x3_2, self.branch7x7x3_3, self.branch7x7x3_4))
        return _cat([b3, b7, Fn.MaxPool3s2Fn.apply(x)])


class InceptionE(nn.Module):
    def __init__(self, in_channels):
        super().__init__()
        self.branch1x1 = BasicConv2d(in_channels, 320, 1)
        self.branch3x3_1 = BasicConv2d(in_channels, 384, 1)
        self.branch3x3_2a = BasicConv2d(384, 384, (1, 3), padding=(0, 1))
        self.branch3x3_2b = BasicConv2d(384, 384, (3, 1), padding=(1, 0))
        self.branch3x3dbl_1 = BasicConv2d(in_channels, 448, 1)
        self.branch3x3dbl_2 = BasicConv2d(448, 384, 3, padding=1)
        self.branch3x3dbl_3a = BasicConv2d(384, 384, (1, 3), padding=(0, 1))
        self.branch3x3dbl_3b = BasicConv2d(384, 384, (3, 1), padding=(1, 0))
        self.branch_pool = BasicConv2d(in_channels, 192, 1)
        self._stem = _Stacked1x1([self.branch1x1, self.branch3x3_1, self.branch3x3dbl_1])

    def forward(self, x):
        b1, b3, td = self._stem(x)
        b3a, b3b = self.branch3x3_2a(b3), self.branch3x3_2b(b3)
        bd = self.branch3x3dbl_2(td, defer=True)  # both consumers gate
        bda, bdb = self.branch3x3dbl_3a(bd, in_relu=True), self.branch3x3dbl_3b(bd, in_relu=True)
        bp = self.branch_pool(Fn.AvgPool3s1Fn.apply(x))
        return _cat([b1, b3a, b3b, bda, bdb, bp])


class CNN_ENCODER(nn.Module):
    """DAMSM.py:117-230: regions (B,256,17,17) from Mixed_6e, code (B,256) from Mixed_7c."""

    def __init__(self, nef, pre_trained=False):
        super().__init__()
        self.nef = 256
        self.Conv2d_1a_3x3 = BasicConv2d(3, 32, 3, stride=2)
        self.Conv2d_2a_3x3 = BasicConv2d(32, 32, 3)
        self.Conv2d_2b_3x3 = BasicConv2d(32, 64, 3, padding=1)
        self.Conv2d_3b_1x1 = BasicConv2d(64, 80, 1)
        self.Conv2d_4a_3x3 = BasicConv2d(80, 192, 3)
        self.Mixed_5b = InceptionA(192, pool_features=32)
        self.Mixed_5c = InceptionA(256, pool_features=64)
        self.Mixed_5d = InceptionA(288, pool_features=64)
        self.Mixed_6a = InceptionB(288)
        self.Mixed_6b = InceptionC(768, channels_7x7=128)
        self.Mixed_6c = InceptionC(768, channels_7x7=160)
        self.Mixed_6d = InceptionC(768, channels_7x7=160)
        self.Mixed_6e = InceptionC(768, channels_7x7=192)
        self.Mixed_7a = InceptionD(768)
        self.Mixed_7b = InceptionE(1280)
        self.Mixed_7c = InceptionE(2048)
        self.emb_features = conv1x1(768, self.nef)
        self.emb_cnn_code = Linear(2048, self.nef)
        for p in self.parameters():
            p.requires_grad = False
        self.init_trainable_weights()

    def init_trainable_weights(self):
        self.emb_features.weight.data.uniform_(-0.1, 0.1)
        self.emb_cnn_code.weight.data.uniform_(-0.1, 0.1)

    def forward(self, x):
        x = Fn.BilinearFn.apply(x if x.dtype == torch.bfloat16 else Fn.ImageToNhwcFn.apply(x), 299, 299)
        x = _chain(x, (self.Conv2d_1a_3x3, self.Conv2d_2a_3x3, self.Conv2d_2b_3x3))
        x = Fn.MaxPool3s2Fn.apply(x)
        x = _chain(x, (self.Conv2d_3b_1x1, self.Conv2d_4a_3x3))
        x = Fn.MaxPool3s2Fn.apply(x)
        x = self.Mixed_5b(x)
        x = self.Mixed_5c(x)
        x = self.Mixed_5d(x)
        x = self.Mixed_6a(x)
        x = self.Mixed_6b(x)
        x = self.Mixed_6c(x)
        x = self.Mixed_6d(x)
        x = self.Mixed_6e(x)
        features = x
        x = self.Mixed_7a(x)
        x = self.Mixed_7b(x)
        x = self.Mixed_7c(x)
        x = Fn.GlobalAvgPoolFn.apply(x)
        cnn_code = self.emb_cnn_code(x)
        features = self.emb_features(features, out_f32=True)
        return features, cnn_code
