"""Cross-rank synchronized BatchNorm (API of sync_batchnorm/batchnorm.py).

Training mode always normalises with batch statistics computed by HIP
kernels; with torch.distributed initialised through eegan_hip.dist the
per-channel (sum, sumsq) partials are all-reduced over RCCL (one fp64
message of 2C values per layer) in forward and (sum dxhat, sum dxhat*xhat)
in backward, which is exactly the gradient flowing through the reference's
ReduceAddCoalesced/Broadcast pair (batchnorm.py:90-111).  Numerics follow
the reference: one process -> F.batch_norm (1/sqrt(var+eps),
batchnorm.py:50-53); several -> clamp(var, eps)^-1/2 with running_var from
the unbiased variance (batchnorm.py:113-125).
"""
import torch

from eegan_hip.nn import SyncBatchNorm2d as _SBN

__all__ = ['SynchronizedBatchNorm1d', 'SynchronizedBatchNorm2d', 'SynchronizedBatchNorm3d']


class SynchronizedBatchNorm2d(_SBN):
    def _check_input_dim(self, input):
        if input.dim() != 4:
            raise ValueError('expected 4D input (got {}D input)'.format(input.dim()))


class _ReshapedBN(_SBN):
    """1d/3d variants: folded onto the 4-D NHWC kernel path."""
    _dims = ()

    def forward(self, x, act=None, slope=0.2):
        if x.dim() not in self._dims:
            raise ValueError('expected {}D input (got {}D input)'.format(' or '.join(map(str, self._dims)), x.dim()))
        shape = x.shape
        x4 = x.reshape(shape[0], shape[1], -1, 1)
        y = super().forward(x4, act=act, slope=slope)
        return y.float().reshape(shape) if x.dtype == torch.float32 else y.reshape(shape)


class SynchronizedBatchNorm1d(_ReshapedBN):
    _dims = (2, 3)


class SynchronizedBatchNorm3d(_ReshapedBN):
    _dims = (5,)
