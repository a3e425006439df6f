"""InceptionV3 pool_3 feature network of the FID leg (reference
metrics/FID/inception.py:7-147) on the HIP kernels.

Same constructor, BLOCK_INDEX_BY_DIM / DEFAULT_BLOCK_INDEX, and forward
contract: a list of the selected blocks' outputs for a (B, 3, H, W) fp32 batch
in [0, 1].  The trunk is torchvision's inception_v3 (the reference builds it
with `models.inception_v3`), here the same modules as DAMSM.CNN_ENCODER's
(torchvision key names, so a torchvision inception_v3 state_dict loads with
`model_path`; AuxLogits / fc keys are not used by the FID blocks): block 0
Conv2d_1a/2a/2b + max pool, block 1 Conv2d_3b/4a + max pool, block 2
Mixed_5b..6e, block 3 Mixed_7a..7c + adaptive average pool.  The input resize
(bilinear, align_corners=True, to 299) and the ImageNet re-normalisation are
one HIP pass (eegan_fid_preprocess).  Block outputs are returned as fp32 NCHW
tensors (the pooled block 3 as (B, 2048, 1, 1)).

Pretrained weights are a network download in the reference
(`models.inception_v3(pretrained=True)`, inception.py:63) and are absent here:
without `model_path` the weights are torchvision's initialisation layout with
seeded random values, so FID values are "parity unpinned" until real weights
are supplied.
"""
import ctypes

import torch
import torch.nn as nn

import DAMSM as _D
from eegan_hip import functional as Fn
from eegan_hip._lib import ops
from eegan_hip.tensor import empty_nhwc, stream

_MEAN = (0.485, 0.456, 0.406)
_STD = (0.229, 0.224, 0.225)


def _to_nchw_f32(x):
    if x.dtype == torch.float32 and x.is_contiguous():
        return x
    return x.float().contiguous()


class InceptionV3(nn.Module):
    """Pretrained InceptionV3 network returning feature maps."""

    DEFAULT_BLOCK_INDEX = 3
    BLOCK_INDEX_BY_DIM = {64: 0, 192: 1, 768: 2, 2048: 3}

    def __init__(self, model_path=None, output_blocks=[DEFAULT_BLOCK_INDEX], resize_input=True,
                 normalize_input=True, requires_grad=False):
        super().__init__()
        self.resize_input = resize_input
        self.normalize_input = normalize_input
        self.output_blocks = sorted(output_blocks)
        self.last_needed_block = max(output_blocks)
        assert self.last_needed_block <= 3, 'Last possible output block index is 3'
        B = _D.BasicConv2d
        self.Conv2d_1a_3x3 = B(3, 32, 3, stride=2)
        self.Conv2d_2a_3x3 = B(32, 32, 3)
        self.Conv2d_2b_3x3 = B(32, 64, 3, padding=1)
        if self.last_needed_block >= 1:
            self.Conv2d_3b_1x1 = B(64, 80, 1)
            self.Conv2d_4a_3x3 = B(80, 192, 3)
        if self.last_needed_block >= 2:
            self.Mixed_5b = _D.InceptionA(192, pool_features=32)
            self.Mixed_5c = _D.InceptionA(256, pool_features=64)
            self.Mixed_5d = _D.InceptionA(288, pool_features=64)
            self.Mixed_6a = _D.InceptionB(288)
            self.Mixed_6b = _D.InceptionC(768, channels_7x7=128)
            self.Mixed_6c = _D.InceptionC(768, channels_7x7=160)
            self.Mixed_6d = _D.InceptionC(768, channels_7x7=160)
            self.Mixed_6e = _D.InceptionC(768, channels_7x7=192)
        if self.last_needed_block >= 3:
            self.Mixed_7a = _D.InceptionD(768)
            self.Mixed_7b = _D.InceptionE(1280)
            self.Mixed_7c = _D.InceptionE(2048)
        if model_path is not None:
            sd = torch.load(model_path, map_location='cpu', weights_only=True)
            own = self.state_dict()
            missing = [k for k in own if k not in sd]
            if missing:
                raise KeyError('%s lacks inception_v3 keys, e.g. %s' % (model_path, missing[:3]))
            self.load_state_dict({k: sd[k] for k in own})
        for p in self.parameters():
            p.requires_grad = requires_grad
        self.eval()

    def _blocks(self):
        blocks = [lambda x: Fn.MaxPool3s2Fn.apply(_D._chain(x, (self.Conv2d_1a_3x3, self.Conv2d_2a_3x3,
                                                               self.Conv2d_2b_3x3)))]
        if self.last_needed_block >= 1:
            blocks.append(lambda x: Fn.MaxPool3s2Fn.apply(_D._chain(x, (self.Conv2d_3b_1x1, self.Conv2d_4a_3x3))))
        if self.last_needed_block >= 2:
            def b2(x):
                for m in (self.Mixed_5b, self.Mixed_5c, self.Mixed_5d, self.Mixed_6a, self.Mixed_6b, self.Mixed_6c,
                          self.Mixed_6d, self.Mixed_6e):
                    x = m(x)
                return x
            blocks.append(b2)
        if self.last_needed_block >= 3:
            blocks.append(lambda x: Fn.GlobalAvgPoolFn.apply(self.Mixed_7c(self.Mixed_7b(self.Mixed_7a(x)))))
        return blocks

    def input_affine(self):
        """Per-channel (scale, shift) of the input re-normalisation (inception.py:135-138)."""
        if self.normalize_input:
            return [s / 0.5 for s in _STD], [(m - 0.5) / 0.5 for m in _MEAN]
        return [1.0] * 3, [0.0] * 3

    def preprocess(self, inp):
        """inception.py:131-138: resize to 299 (bilinear, align_corners=True) and
        re-normalise to the ImageNet statistics, as one HIP pass -> NHWC bf16."""
        x = _to_nchw_f32(inp)
        N, C, H, W = x.shape
        if C != 3:
            raise ValueError('InceptionV3 expects 3-channel input')
        Ho, Wo = (299, 299) if self.resize_input else (H, W)
        sc, sh = self.input_affine()
        y = empty_nhwc(N, 3, Ho, Wo, x.device)
        F3 = ctypes.c_float * 3
        ops.fid_preprocess(x.data_ptr(), N, H, W, Ho, Wo, F3(*sc), F3(*sh), y.data_ptr(), 8, stream())
        return y

    @torch.no_grad()
    def forward(self, inp):
        return self.forward_prepared(self.preprocess(inp))

    @torch.no_grad()
    def forward_prepared(self, x):
        """The blocks on an input already resized / re-normalised into NHWC bf16
        (preprocess, or metrics.FID.sampling's generator-sample path)."""
        outp = []
        for idx, block in enumerate(self._blocks()):
            x = block(x)
            if idx in self.output_blocks:
                if x.dim() == 2:   # the pooled block 3: (B, 2048) -> (B, 2048, 1, 1)
                    outp.append(x.reshape(x.shape[0], -1, 1, 1))
                else:
                    outp.append(x.float().contiguous())
            if idx == self.last_needed_block:
                break
        return outp
