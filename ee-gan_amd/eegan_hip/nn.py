"""Parameter-holding modules with the exact parameter/buffer names of
torch.nn.Conv2d / nn.Linear / the reference's SynchronizedBatchNorm2d, so
state_dicts of the reference load unchanged.  Their forward passes run on
libeegan_hip.so through eegan_hip.functional."""
import math

import torch
import torch.nn as nn

from . import functional as Fn
from ._lib import ACT_CODES
from .tensor import to_nhwc_bf16


def _pair(v):
    return (v, v) if isinstance(v, int) else tuple(v)


class Conv2d(nn.Module):
    """nn.Conv2d-compatible (weight (Cout,Cin,kh,kw) stored channels-last, optional bias).
    forward(x, act=None, slope=0.2, out_f32=False, up2=False, in_act=None, defer_act=False):
    the activation is fused into the epilogue and up2 reads x through a
    nearest-2x upsample; in_act / defer_act fuse an activation's backward
    into the consuming conv's data gradient (Fn.Conv2dFn)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, bias=True):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.kernel_size = _pair(kernel_size)
        self.stride = stride if isinstance(stride, int) else stride[0]
        self.padding = _pair(padding)
        # channels-last storage ([Cout][kh][kw][Cin], torch.channels_last): the layout
        # the kernels pack from and write weight gradients into with unit stride
        self.weight = nn.Parameter(torch.empty(out_channels, in_channels, *self.kernel_size).contiguous(
            memory_format=torch.channels_last))
        self.bias = nn.Parameter(torch.empty(out_channels)) if bias else None
        self.reset_parameters()
        self._cache = Fn.PackCache()
        self._geo = {}

    def reset_parameters(self):  # nn.Conv2d's default init
        nn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        if self.bias is not None:
            fan_in = self.weight.shape[1] * self.kernel_size[0] * self.kernel_size[1]
            bound = 1 / math.sqrt(fan_in) if fan_in > 0 else 0
            nn.init.uniform_(self.bias, -bound, bound)

    def geom(self, up2=False):
        g = self._geo.get(up2)
        if g is None:
            g = Fn.Geom(self.out_channels, self.kernel_size[0], self.kernel_size[1], self.stride, self.padding[0],
                        self.padding[1], int(up2))
            self._geo[up2] = g
        return g

    def forward(self, x, act=None, slope=0.2, out_f32=False, up2=False, in_act=None, in_slope=0.2,
                defer_act=False):
        """in_act / defer_act: fused activation backward across a single-consumer
        link (see Fn.Conv2dFn)."""
        return Fn.Conv2dFn.apply(x, self.weight, self.bias, self.geom(up2), ACT_CODES[act], slope, out_f32,
                                 self._cache, ACT_CODES[in_act], in_slope, defer_act)

    def extra_repr(self):
        return '%d, %d, kernel_size=%s, stride=%d, padding=%s, bias=%s' % (
            self.in_channels, self.out_channels, self.kernel_size, self.stride, self.padding, self.bias is not None)


class Linear(nn.Module):
    """nn.Linear-compatible fp32 linear (forward(x, act=None))."""

    def __init__(self, in_features, out_features, bias=True):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.weight = nn.Parameter(torch.empty(out_features, in_features))
        self.bias = nn.Parameter(torch.empty(out_features)) if bias else None
        nn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        if self.bias is not None:
            bound = 1 / math.sqrt(in_features) if in_features > 0 else 0
            nn.init.uniform_(self.bias, -bound, bound)

    def forward(self, x, act=None):
        return Fn.LinearFn.apply(x, self.weight, self.bias, ACT_CODES[act])


class SyncBatchNorm2d(nn.Module):
    """Buffers/params of sync_batchnorm.SynchronizedBatchNorm2d (batchnorm.py:38-46,
    191-251): weight/bias (affine), running_mean/var, num_batches_tracked.
    Training mode always uses batch statistics, synchronised across ranks when
    torch.distributed is initialised through eegan_hip.dist (RCCL all-reduce of
    (sum, sumsq) in forward and (sum dxhat, sum dxhat*xhat) in backward)."""

    def __init__(self, num_features, eps=1e-5, momentum=0.1, affine=True):
        super().__init__()
        self.num_features, self.eps, self.momentum, self.affine = num_features, eps, momentum, affine
        self.track_running_stats = True
        if affine:
            self.weight = nn.Parameter(torch.ones(num_features))
            self.bias = nn.Parameter(torch.zeros(num_features))
        else:
            self.register_parameter('weight', None)
            self.register_parameter('bias', None)
        self.register_buffer('running_mean', torch.zeros(num_features))
        self.register_buffer('running_var', torch.ones(num_features))
        self.register_buffer('num_batches_tracked', torch.tensor(0, dtype=torch.long))
        # replication state (batchnorm.py:42-46), set by sync_batchnorm.replicate's callbacks
        self._is_parallel = False
        self._parallel_id = None
        self._sync_group = None

    def __data_parallel_replicate__(self, ctx, copy_id):
        """batchnorm.py:80-88: copy 0 is the master.  One process per GPU: the
        copies are the ranks, and ctx.sync_master is the rank group whose
        transport (eegan_hip.dist: RCCL or the peer-write kernel) carries the
        statistics; the kernels synchronise whenever it spans more than one
        rank, which is when the reference leaves F.batch_norm (batchnorm.py:50)."""
        self._parallel_id = copy_id
        self._sync_group = getattr(ctx, 'sync_master', None)
        self._is_parallel = self._sync_group is not None and self._sync_group.world > 1

    def forward(self, x, act=None, slope=0.2, up2=False):
        if not self.training:
            return self._eval_forward(x, act, slope, up2)
        return Fn.BnModFn.apply(x, self.weight, self.bias, None, None, None, self, 0, ACT_CODES[act], slope, up2)

    def modulate(self, x, gam, bet, mask, act=None, slope=0.2, up2=False):
        """affine_ssa: act((gam*m + 1) * BN(x) + bet*m) (models.py:69-86)."""
        return Fn.BnModFn.apply(x, None, None, gam, bet, mask, self, 1, ACT_CODES[act], slope, up2)

    def _eval_forward(self, x, act, slope, up2):
        # running statistics: the normalisation is a per-channel affine map
        w = self.weight if self.weight is not None else torch.ones_like(self.running_mean)
        b = self.bias if self.bias is not None else torch.zeros_like(self.running_mean)
        scale = w / torch.sqrt(self.running_var + self.eps)
        shift = b - self.running_mean * scale
        return Fn.BnEvalFn.apply(x, scale.float().contiguous(), shift.float().contiguous(), ACT_CODES[act], slope,
                                 up2)
