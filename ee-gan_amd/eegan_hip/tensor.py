"""NHWC tensor helpers.

Activations are torch tensors with the LOGICAL shape (N, C, H, W) of the
reference but channels-last storage with a channel stride `ld`
(ld == C for C < 8, else a multiple of 8 >= C) and dtype bfloat16.  Torch is
only the allocator/stream provider here; all arithmetic runs in
libeegan_hip.so.
"""
import torch

from ._lib import ops

BF16 = torch.bfloat16
F32 = torch.float32
CL = torch.channels_last  # fp32 conv weights: (Cout, Cin, R, S) stored [Cout][R][S][Cin]


def ld_for(C, dtype=BF16):
    """bf16 activations: channel stride rounded up to 8 (16-byte pixel rows, so
    even 3-channel images feed the vectorised gathers); fp32 tensors: dense."""
    if dtype != BF16:
        return C
    return (C + 7) // 8 * 8


def stream():
    return torch.cuda.current_stream().cuda_stream


def empty_nhwc(N, C, H, W, device, dtype=BF16, ld=None):
    ld = ld_for(C, dtype) if ld is None else ld
    buf = torch.empty((N, H, W, ld), dtype=dtype, device=device)
    if ld != C:
        buf = buf[..., :C]
    return buf.permute(0, 3, 1, 2)


def ld_of(t):
    """Channel stride of an NHWC-stored (N, C, H, W) tensor (robust to size-1 dims)."""
    N, C, H, W = t.shape
    if W > 1:
        return t.stride(3)
    if H > 1:
        return t.stride(2)
    if N > 1:
        return t.stride(0)
    return ld_for(C, t.dtype)


def is_nhwc(t):
    """NHWC-stored activation usable by the kernels: bf16 needs ld % 8 == 0
    and a 16-byte aligned base; fp32 is accepted dense or padded."""
    if t.dim() != 4 or t.stride(1) != 1 and t.shape[1] > 1:
        return False
    N, C, H, W = t.shape
    ld = ld_of(t)
    if ld < C:
        return False
    if t.dtype == BF16 and (ld % 8 or t.data_ptr() % 16):
        return False
    if W > 1 and t.stride(3) != ld:
        return False
    if H > 1 and t.stride(2) != W * ld:
        return False
    if N > 1 and t.stride(0) != H * W * ld:
        return False
    return True


def to_nhwc_bf16(t):
    """Return `t` unchanged when it already is an NHWC bf16 activation, else a
    converted copy (fp32 NCHW -> HIP conversion kernel)."""
    if t.dtype == BF16 and is_nhwc(t):
        return t
    if t.dtype == F32 and t.is_contiguous():
        N, C, H, W = t.shape
        out = empty_nhwc(N, C, H, W, t.device)
        ops.nchw_to_nhwc(t.data_ptr(), N, C, H * W, out.data_ptr(), ld_of(out), stream())
        return out
    N, C, H, W = t.shape
    out = empty_nhwc(N, C, H, W, t.device, dtype=t.dtype if t.dtype in (BF16, F32) else BF16)
    out.copy_(t)  # rare layout repair (e.g. autograd-summed padded views)
    if out.dtype != BF16:
        return to_nhwc_bf16(out.contiguous())
    return out


def ptr(t):
    return 0 if t is None else t.data_ptr()


def new_stream(device, priority=0):
    """A HIP stream of its own (never recycled: torch.cuda.Stream() hands out
    pool streams round-robin, so after 32 of them two "different" streams can
    be one HIP stream and lanes meant to overlap -- or a lane and a capture
    stream -- alias).  Lives for the process.  priority > 0: the device's
    highest stream priority, < 0 its lowest."""
    import ctypes
    from ._lib import ops
    h = ctypes.c_void_p()
    ops.stream_create(ctypes.byref(h), int(priority))
    return torch.cuda.ExternalStream(h.value, device=device)


def workspace(nbytes, device):
    return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=device)
