"""torch.autograd.Functions over libeegan_hip.so.

Every Function launches HIP kernels through the C ABI on torch's current
stream; torch provides memory (caching allocator), streams and the autograd
tape.  The discriminator-side Functions (conv, activation, avg-pool,
scale-add, cat-tile, cast) express their backward through other Functions,
so they are differentiable to any order -- needed by the MA gradient penalty
(train.py:378-402, autograd.grad(create_graph=True) through every D layer).
Generator-side Functions (BN modulation, upsample-fused convs, linears,
mask resize) are first-order, as the reference only differentiates G once.
"""
import ctypes
import contextlib
import os
import math

import torch

from . import tensor as T
from ._lib import ops, ConvDesc, BnModDesc, GemmDesc, ACT_CODES
from .tensor import BF16, F32, CL, empty_nhwc, ld_of, ptr, stream, to_nhwc_bf16, workspace

# In autograd.grad() mode the engine cannot report whether a leaf is needed;
# parameters are then assumed NOT requested (the gradient penalty asks only
# for input gradients: train.py:389-394).  Set False to always compute them.
SKIP_PARAM_GRADS_IN_AUTOGRAD_GRAD = True

# Process-group hook for SyncBN statistics (set by eegan_hip.dist)
SYNC_BN_ALLREDUCE = None   # callable(tensor fp64) -> None (in-place sum over ranks)
SYNC_BN_WORLD = 1
# The reference's multi-device numerics (clamp(var, eps)^-1/2, zero gradient
# through the clamp, running_var from the unbiased variance:
# sync_batchnorm/batchnorm.py:113-125) are used whenever the world is > 1;
# EEGAN_SYNCBN_MULTI=1 (or this flag) selects them at world 1 too, so one GPU
# can test the kernels' clamp path against the oracle's restatement.
SYNC_BN_FORCE_MULTI = os.environ.get('EEGAN_SYNCBN_MULTI', '0') == '1'


def _syncbn_world():
    """World size of the SyncBN statistics.  A process group started by the
    caller (reference train.py under torchrun, not eegan_hip.dist.init_from_env)
    is picked up on first use, so the drop-in modules synchronise without any
    call into this package."""
    if SYNC_BN_ALLREDUCE is None:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            from . import dist as D
            D.install_syncbn_hook()
    return SYNC_BN_WORLD


def _needed(ctx, i):
    if not ctx.needs_input_grad[i]:
        return False
    node = ctx.next_functions[i][0]
    if node is None:
        return False
    try:
        return bool(torch._C._will_engine_execute_node(node))
    except RuntimeError:
        var = getattr(node, 'variable', None)
        if SKIP_PARAM_GRADS_IN_AUTOGRAD_GRAD and isinstance(var, torch.nn.Parameter):
            return False
        return True


# When autograd would only add a parameter gradient into an existing fp32
# p.grad (FlatAdam keeps p.grad as a view of its flat gradient buffer), the
# kernels accumulate straight into p.grad and the Function returns None for
# it: no temporary dW and no separate add launch.  Off under create_graph
# (the gradient penalty's double backward) and for non-leaf inputs.
DIRECT_PARAM_GRADS = True


_PENDING_SINKS = set()   # FlatAdam objects holding buckets completed by this Function's writes


def _commit_sinks():
    """After a Function's backward has launched its kernels: issue the
    all-reduces of the buckets its direct gradient writes completed (same
    stream, so they follow the writes)."""
    while _PENDING_SINKS:
        _PENDING_SINKS.pop().flush_ready()


def _grad_sink(ctx, i):
    g = _sink_of(ctx, i)
    var = getattr(ctx.next_functions[i][0], 'variable', None) if ctx.next_functions[i][0] is not None else None
    tr = getattr(var, '_eegan_track', None) if var is not None else None
    if tr is not None:   # FlatAdam's overlapped all-reduce counts the writes
        if g is not None:
            if tr.note_grad_write(var, type(ctx).__name__):
                _PENDING_SINKS.add(tr)
        else:
            tr.note_autograd_write(var)   # this gradient goes through autograd's accumulation instead
    return g


def _sink_of(ctx, i):
    if not DIRECT_PARAM_GRADS or torch.is_grad_enabled():
        return None
    node = ctx.next_functions[i][0]
    var = getattr(node, 'variable', None)
    if var is None or getattr(var, '_eegan_hooked', False):
        return None   # hooked parameters (eegan_hip.dist.GradHooks) need AccumulateGrad to run
    g = var.grad
    if g is None or g.dtype != F32 or g.shape != var.shape or g.stride() != var.stride():
        return None
    if g.dim() == 4 and not g.is_contiguous(memory_format=CL):
        return None   # conv weight gradients are written channels-last only
    return g


def _sink_wgrad(ctx, i, x, dz, g, W_shape):
    """dW of input i accumulated into its FlatAdam gradient view; False when
    the gradient has to go through autograd instead."""
    sink = _grad_sink(ctx, i)
    if sink is None or not sink.is_contiguous(memory_format=CL):
        return False
    conv_bwd_weight_raw(x, dz, g, W_shape, out=sink)
    return True


def _sink_chansum(ctx, i, dz, sink):
    chansum_raw(dz, out=sink)


# ============================================================== weights ===
class PackCache:
    """bf16 packed images of one conv weight (forward and bwd-data layouts),
    rebuilt whenever the fp32 parameter changes (torch in-place version or
    the flat-Adam generation counter).  Rebuilds write into the SAME buffer:
    a captured step graph keeps reading the address it captured, so a pack
    refreshed later in the step (or by the next replay) must land there."""

    def __init__(self, scale=None):
        self.fwd_key = self.bwd_key = None
        self.fwd = self.bwd = None
        self.scale = scale  # optional per-output-channel fp32 scale folded into the packs

    @staticmethod
    def _key(W):
        gen = getattr(W, '_eegan_gen', None)
        return (W.data_ptr(), W._version, gen[0] if gen is not None else 0)

    def get(self, W, transposed):
        W._eegan_packcache = self   # FlatAdam re-packs registered weights in one launch after its step
        key = self._key(W)
        if transposed:
            if self.bwd_key != key:
                self.bwd = pack_weight(W, True, self.scale, out=self.bwd)
                self.bwd_key = key
            return self.bwd
        if self.fwd_key != key:
            self.fwd = pack_weight(W, False, self.scale, out=self.fwd)
            self.fwd_key = key
        return self.fwd


def pack_weight(W, transposed, scale=None, out=None):
    Cout, Cin, R, S = W.shape
    n = ops.conv_packed_elems(Cout, Cin, R, S, int(transposed))
    if out is None or out.numel() != n or out.device != W.device:
        out = torch.empty(n, dtype=BF16, device=W.device)
    Wc = W.detach()
    if Wc.dtype != F32 or not Wc.is_contiguous(memory_format=CL):
        Wc = Wc.float().contiguous(memory_format=CL)
    ops.conv_pack_weights(Wc.data_ptr(), ptr(scale), Cout, Cin, R, S, int(transposed), out.data_ptr(), stream())
    return out


def _pack(W, cache, transposed):
    if cache is not None:
        return cache.get(W, transposed)
    return pack_weight(W, transposed)


class Geom:
    """Static conv geometry (per module); the batch/grid sizes come from x."""
    __slots__ = ('K', 'R', 'S', 'stride', 'ph', 'pw', 'up2')

    def __init__(self, K, R, S, stride, ph, pw, up2=0):
        self.K, self.R, self.S, self.stride, self.ph, self.pw, self.up2 = K, R, S, stride, ph, pw, up2

    def out_hw(self, H, W):
        Hl, Wl = (H * 2, W * 2) if self.up2 else (H, W)
        return ((Hl + 2 * self.ph - self.R) // self.stride + 1, (Wl + 2 * self.pw - self.S) // self.stride + 1)

    def desc(self, x, ldy):
        N, C, H, W = x.shape
        Ho, Wo = self.out_hw(H, W)
        Hl, Wl = (H * 2, W * 2) if self.up2 else (H, W)
        return ConvDesc(N, Hl, Wl, C, ld_of(x), self.K, self.R, self.S, self.stride, self.ph, self.pw, self.up2,
                        Ho, Wo, ldy)


# Split-K counters (eegan_conv_desc.splitk_ctr): one zeroed int array per stream, so
# the kernels finish a split-K launch themselves (csrc/conv.hip splitk_fused_finish;
# every counter used is zero again when the launch completes) and launches on
# different stream lanes never share a counter.  Created outside graph capture (the
# step's eager warm-up reaches every lane first); a stream first seen inside a
# capture keeps the two-launch reduce.  SPLITK_FUSED = False: always two launches.
# The library uses the counters only with EEGAN_CONV splitk_fused=1: on the replayed
# C2 step the in-kernel finish measured -0.7 % against the separate reduce launch
# (in-process A/B, profiles/r05_inproc_ab.txt), so the reduce launch is the default
# and no counters are allocated unless both switches are on (EEGAN_SPLITK_FUSED=1).
SPLITK_FUSED = os.environ.get('EEGAN_SPLITK_FUSED', '0') == '1'
SPLITK_CTR_N = 1 << 15
_SPLITK_CTR = {}


def _splitk_ctr(device):
    if not SPLITK_FUSED:
        return None
    s = torch.cuda.current_stream(device).cuda_stream
    t = _SPLITK_CTR.get((device, s))
    if t is None:
        if torch.cuda.is_current_stream_capturing():
            return None
        t = _SPLITK_CTR[(device, s)] = torch.zeros(SPLITK_CTR_N, dtype=torch.int32, device=device)
    return t


# Planner objective per stream (eegan_conv_desc.plan): cuda_stream handle -> 1 for
# the step's lanes that run beside the critical chain (trainer.TP_LANES), whose
# convs are planned for throughput (larger tiles, no split-K) instead of latency.
# Read when a conv is issued -- inside a graph capture, when the graph is built.
STREAM_PLAN = {}


def _desc_io(g, x_shape, ldx, ldy, device=None):
    N, C, H, W = x_shape
    Hl, Wl = (H * 2, W * 2) if g.up2 else (H, W)
    Ho = (Hl + 2 * g.ph - g.R) // g.stride + 1
    Wo = (Wl + 2 * g.pw - g.S) // g.stride + 1
    d = ConvDesc(N, Hl, Wl, C, ldx, g.K, g.R, g.S, g.stride, g.ph, g.pw, g.up2, Ho, Wo, ldy)
    if STREAM_PLAN:
        d.plan = STREAM_PLAN.get(torch.cuda.current_stream().cuda_stream, 0)
    if device is not None and device.type == 'cuda':
        ctr = _splitk_ctr(device)
        if ctr is not None:
            d.splitk_ctr, d.splitk_ctr_n = ctr.data_ptr(), ctr.numel()
    return d


# ====================================================== launch timing ====
class LaunchTimer(object):
    """Times every launch of the conv / linear GEMM kernels (bench.py's
    roofline): each op is armed with HIP timing events that its kernels
    (the GEMM and, with split-K, its reduce) take through hipExtLaunchKernel,
    so the events carry the dispatches' own begin/end stamps on the stream
    they run on, with no host launch gap inside.  Records (kind, algorithmic
    flops, algorithmic bytes, [(start, stop), ...]).  Not usable inside a
    graph capture (bench.py times an eager pass of the same step)."""

    def __init__(self, detail=False):
        self.rec = []
        self.detail = detail
        self._pool = []
        self.ops = []   # issue order: (kind, shape key, flops, bytes, dispatches) -- tools/rocprof_families.py --ops

    def _event(self):
        ev = ctypes.c_void_p()
        ops.event_create(ctypes.byref(ev))
        self._pool.append(ev)
        return ev

    def __call__(self, kind, flops, nbytes, fn, key=None):
        ev = [self._event() for _ in range(4)]
        ops.timing_arm(*ev)
        try:
            fn()
        finally:
            n = ctypes.c_int()
            ops.timing_disarm(ctypes.byref(n))
        self.rec.append((kind if not self.detail else (kind, key), flops, nbytes,
                         [(ev[2 * i], ev[2 * i + 1]) for i in range(n.value)]))
        self.ops.append((kind, key, flops, nbytes, n.value))

    def summary(self):
        """{kind: [launches, flops, bytes, seconds]} (seconds = summed kernel time)."""
        torch.cuda.synchronize()
        out = {}
        ms = ctypes.c_float()
        for kind, fl, nb, pairs in self.rec:
            t = 0.0
            for e0, e1 in pairs:
                ops.event_elapsed(e0, e1, ctypes.byref(ms))
                t += ms.value * 1e-3
            o = out.setdefault(kind, [0, 0.0, 0.0, 0.0])
            o[0] += 1
            o[1] += fl
            o[2] += nb
            o[3] += t
        return out

    def __del__(self):
        for ev in getattr(self, '_pool', []):
            try:
                ops.event_destroy(ev)
            except Exception:
                pass


TIMER = None

# Phase stamps (diagnostics, tools/stamp_phases.py): when STAMPS is a list,
# stamp(name) launches a one-thread kernel writing the device clock into the
# next slot of STAMP_BUF on the current stream -- it survives graph capture,
# so phase durations of a replayed step can be read back.
STAMPS = None
STAMP_BUF = None


def stamp(name):
    if STAMPS is None:
        return
    i = len(STAMPS)
    if i >= STAMP_BUF.numel():
        raise RuntimeError('stamp buffer full')
    STAMPS.append((name, torch.cuda.current_stream().cuda_stream))
    ops.stamp(STAMP_BUF.data_ptr() + 8 * i, stream())


def _launch(kind, flops, nbytes, fn, key=None):
    if TIMER is None:
        fn()
    else:
        TIMER(kind, flops, nbytes, fn, key)


def _shape_key(d):
    return 'N%d %dx%d C%d->K%d %dx%d s%d p%d,%d%s -> %dx%d' % (d.N, d.H, d.W, d.C, d.K, d.R, d.S, d.stride, d.pad_h,
                                                             d.pad_w, ' up2' if d.up2 else '', d.Ho, d.Wo)


# ============================================================ conv core ===
def conv_fwd_raw(x, W, b, g, act=0, slope=0.2, out_f32=False, cache=None, res=None, gamma=None):
    x = to_nhwc_bf16(x)
    N, C, H, Wd = x.shape
    Ho, Wo = g.out_hw(H, Wd)
    y = empty_nhwc(N, g.K, Ho, Wo, x.device, dtype=F32 if out_f32 else BF16)
    d = _desc_io(g, x.shape, ld_of(x), ld_of(y), x.device)
    wp = _pack(W, cache, False)
    wsb = ops.conv_fwd_workspace(d)
    ws = workspace(wsb, x.device) if wsb else None
    flops = 2.0 * N * Ho * Wo * g.K * C * g.R * g.S
    nbytes = 2.0 * (N * H * Wd * C + N * Ho * Wo * g.K * (2 if out_f32 else 1) + g.K * C * g.R * g.S)
    _launch('conv_fwd', flops, nbytes, lambda: ops.conv_fwd(
        d, x.data_ptr(), wp.data_ptr(), ptr(b), act, slope, ptr(res), ld_of(res) if res is not None else 0,
        ptr(gamma), y.data_ptr(), int(out_f32), ptr(ws), stream()), key=_shape_key(d) if TIMER is not None else None)
    return y


def conv_bwd_data_raw(dz, W, g, x_shape, cache=None, gate=None, gate_act=0, gate_slope=0.2, res=None, res_up2=0,
                      res_scale=1.0):
    """dx for the LOGICAL input grid (hi-res when g.up2), NHWC bf16.  `gate`
    (the activated conv input, act code gate_act): dx *= act'(gate) in the
    epilogue -- the producing layer's activation backward, fused."""
    if (gate is not None or res is not None) and g.up2:
        raise ValueError('conv_bwd_data_raw: gated / residual data gradients of up2 convs are not supported')
    N, C, H, Wd = x_shape
    Hl, Wl = (H * 2, Wd * 2) if g.up2 else (H, Wd)
    dx = empty_nhwc(N, C, Hl, Wl, dz.device)
    dz = to_nhwc_bf16(dz)
    d = _desc_io(g, x_shape, T.ld_for(C), ld_of(dz), dz.device)
    if g.up2:
        d.H, d.W, d.up2 = Hl, Wl, 0
    wp = _pack(W, cache, True)
    wsb = ops.conv_bwd_data_workspace(d)
    ws = workspace(wsb, dz.device) if wsb else None
    Ho, Wo = d.Ho, d.Wo
    flops = 2.0 * N * Ho * Wo * g.K * C * g.R * g.S
    nbytes = 2.0 * (N * Hl * Wl * C + N * Ho * Wo * g.K + g.K * C * g.R * g.S)
    if res is not None:
        _launch('conv_bwd_data', flops, nbytes, lambda: ops.conv_bwd_data_ex(
            d, dz.data_ptr(), wp.data_ptr(), dx.data_ptr(), ld_of(dx), 0, ptr(gate),
            ld_of(gate) if gate is not None else 0, gate_act, gate_slope, res.data_ptr(), ld_of(res), int(res_up2),
            res_scale, ptr(ws), stream()), key=_shape_key(d) if TIMER is not None else None)
    elif gate is None:
        _launch('conv_bwd_data', flops, nbytes, lambda: ops.conv_bwd_data(
            d, dz.data_ptr(), wp.data_ptr(), dx.data_ptr(), ld_of(dx), 0, ptr(ws), stream()),
            key=_shape_key(d) if TIMER is not None else None)
    else:
        _launch('conv_bwd_data', flops, nbytes, lambda: ops.conv_bwd_data_gated(
            d, dz.data_ptr(), wp.data_ptr(), dx.data_ptr(), ld_of(dx), 0, gate.data_ptr(), ld_of(gate), gate_act,
            gate_slope, ptr(ws), stream()), key=_shape_key(d) if TIMER is not None else None)
    if g.up2:
        lo = empty_nhwc(N, C, H, Wd, dz.device)
        ops.sumpool2(dx.data_ptr(), N, Hl, Wl, C, ld_of(dx), lo.data_ptr(), ld_of(lo), stream())
        return lo
    return dx


def conv_bwd_weight_raw(x, dz, g, W_shape, out=None):
    """dW (fresh channels-last fp32 tensor), or accumulated into `out` when given."""
    x = to_nhwc_bf16(x)
    d = _desc_io(g, x.shape, ld_of(x), ld_of(dz))
    ws = workspace(ops.conv_wgrad_workspace(d), x.device)
    if out is not None and not out.is_contiguous(memory_format=CL):
        raise ValueError('conv_bwd_weight: dW accumulates into channels-last fp32 storage')
    dW = torch.empty(W_shape, dtype=F32, device=x.device, memory_format=CL) if out is None else out
    N, C, H, Wd = x.shape
    flops = 2.0 * N * d.Ho * d.Wo * g.K * C * g.R * g.S
    nbytes = 2.0 * (N * H * Wd * C + N * d.Ho * d.Wo * g.K) + 4.0 * g.K * C * g.R * g.S
    _launch('conv_bwd_weight', flops, nbytes, lambda: ops.conv_bwd_weight(
        d, x.data_ptr(), dz.data_ptr(), ws.data_ptr(), dW.data_ptr(), int(out is not None), stream()),
        key=_shape_key(d) if TIMER is not None else None)
    return dW


def chansum_raw(dz, out=None):
    N, C, H, W = dz.shape
    P = N * H * W
    ws = workspace(ops.chansum_workspace(P, C), dz.device)
    acc = out is not None
    if out is None:
        out = torch.empty(C, dtype=F32, device=dz.device)
    ops.chansum(dz.data_ptr(), ld_of(dz), P, C, ws.data_ptr(), out.data_ptr(), int(acc), stream())
    return out


def act_bwd_raw(gy, y, act, slope):
    N, C, H, W = y.shape
    dx = empty_nhwc(N, C, H, W, y.device)
    ops.act_bwd(gy.data_ptr(), ld_of(gy), y.data_ptr(), ld_of(y), N * H * W, C, act, slope, dx.data_ptr(), ld_of(dx),
                stream())
    return dx


def _as_bf16_grad(g):
    if g.dtype == F32:
        return CastF32Bf16Fn.apply(g)
    return to_nhwc_bf16(g)


# EEGAN_FUSE_ACT_BWD=0: every activation backward runs as its own pass (A/B switch).
FUSE_ACT_BWD = os.environ.get('EEGAN_FUSE_ACT_BWD', '1') != '0'
# False: under create_graph (the gradient penalty's first backward) every
# activation backward runs as its own ActBwdFn pass (module constant for A/B:
# tools/ab_inproc.py "py:eegan_hip.functional.FUSE_GP_ACT=False").
FUSE_GP_ACT = True


def _act_deferred(ctx, fused, cg):
    """Whether this layer's activation backward runs in its consumers instead.
    defer_act=True: every consumer is a conv with in_act (gates in the first-
    order backward and, through GatedConvBwdDataFn, under create_graph);
    defer_act='first_order': the consumer gates in the first-order backward
    and, with FUSE_GP_GATE, under create_graph too (resD's ScaleAddFn h_act:
    ScaleAddGateBwdFn)."""
    return bool(ctx.defer_act) and (fused or (cg and (ctx.defer_act is True or FUSE_GP_GATE)))


class Conv2dFn(torch.autograd.Function):
    """y = act(conv(x, W) + b); NHWC bf16 in, bf16 (or fp32) out.

    Activation backward fused across a single-consumer link (first-order
    backward only; under create_graph both sides fall back to ActBwdFn):
    `in_act` = activation that produced x (x = act(z) of a layer called with
    `defer_act=True`): dx is multiplied by act'(x) in the data-gradient
    epilogue, and the producer passes its incoming gradient on unmasked.  The
    factor distributes over a sum of gradients, so x may have several
    consumers as long as every one of them gates (models decide: resD,
    DiscSent/DiscCond heads, Inception branch chains)."""

    @staticmethod
    def forward(ctx, x, W, b, g, act, slope, out_f32, cache, in_act=0, in_slope=0.2, defer_act=False):
        x = to_nhwc_bf16(x)
        if in_act and g.up2:
            raise ValueError('Conv2dFn: in_act with up2 is not supported')
        y = conv_fwd_raw(x, W, b, g, act, slope, out_f32, cache)
        ctx.g, ctx.act, ctx.slope, ctx.cache = g, act, slope, cache
        ctx.in_act, ctx.in_slope, ctx.defer_act = in_act, in_slope, defer_act
        ctx.x_shape = tuple(x.shape)
        ctx.save_for_backward(x, W, y if act else None)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, W, y = ctx.saved_tensors
        g = ctx.g
        gy = _as_bf16_grad(gy)
        fused = FUSE_ACT_BWD and not torch.is_grad_enabled()
        cg = FUSE_ACT_BWD and FUSE_GP_ACT and torch.is_grad_enabled()
        dz = (ActBwdFn.apply(gy, _mask_src(y, ctx.act), ctx.act, ctx.slope)
              if ctx.act and not _act_deferred(ctx, fused, cg) else gy)
        dx = dW = db = None
        if _needed(ctx, 0):
            if g.up2:
                dx = conv_bwd_data_raw(dz, W, g, ctx.x_shape, ctx.cache)
            elif fused and ctx.in_act:
                dx = conv_bwd_data_raw(dz, W, g, ctx.x_shape, ctx.cache, gate=x, gate_act=ctx.in_act,
                                       gate_slope=ctx.in_slope)
            elif cg and ctx.in_act:
                dx = GatedConvBwdDataFn.apply(dz, W, _mask_src(x, ctx.in_act), g, ctx.x_shape, ctx.cache, ctx.in_act,
                                              ctx.in_slope)
            else:
                dx = ConvBwdDataFn.apply(dz, W, g, ctx.x_shape, ctx.cache)
        if _needed(ctx, 1) and not _sink_wgrad(ctx, 1, x, dz, g, W.shape):
            dW = ConvBwdWeightFn.apply(x, dz, g) if not g.up2 else conv_bwd_weight_raw(x, dz, g, W.shape)
        if ctx.needs_input_grad[2] and _needed(ctx, 2):
            sink = _grad_sink(ctx, 2)
            if sink is not None:
                _sink_chansum(ctx, 2, dz, sink)
            else:
                db = ChanSumFn.apply(dz)
        return dx, dW, db, None, None, None, None, None, None, None, None


class PoolConvFn(torch.autograd.Function):
    """(avg_pool2d(x, 2), act(conv(x, W) + b)) of one resD input
    (models.py:267-285: the shortcut pools x, the residual's first conv reads
    x).  The first-order backward returns ONE dx: the conv's data gradient
    with the pooled branch's gradient (x 1/4 at (y/2, x/2)) added in its
    epilogue -- no average-pool adjoint pass, no gradient add.  Under
    create_graph it is composed of the differentiable Functions instead.
    defer_act as in Conv2dFn."""

    @staticmethod
    def forward(ctx, x, W, b, g, act, slope, cache, defer_act=False):
        x = to_nhwc_bf16(x)
        N, C, H, Wd = x.shape
        p = empty_nhwc(N, C, H // 2, Wd // 2, x.device)
        ops.avgpool2(x.data_ptr(), N, H, Wd, C, ld_of(x), p.data_ptr(), ld_of(p), stream())
        y = conv_fwd_raw(x, W, b, g, act, slope, False, cache)
        ctx.g, ctx.act, ctx.slope, ctx.cache, ctx.defer_act = g, act, slope, cache, defer_act
        ctx.x_shape = tuple(x.shape)
        ctx.save_for_backward(x, W, y if act else None)
        return p, y

    @staticmethod
    def backward(ctx, gp, gy):
        x, W, y = ctx.saved_tensors
        g = ctx.g
        fused = FUSE_ACT_BWD and not torch.is_grad_enabled()
        cg = FUSE_ACT_BWD and FUSE_GP_ACT and torch.is_grad_enabled()
        dx = dW = db = None
        dz = None
        if gy is not None:
            gy = _as_bf16_grad(gy)
            dz = (ActBwdFn.apply(gy, _mask_src(y, ctx.act), ctx.act, ctx.slope)
              if ctx.act and not _act_deferred(ctx, fused, cg) else gy)
        if _needed(ctx, 0):
            if fused and gp is not None and dz is not None:
                dx = conv_bwd_data_raw(dz, W, g, ctx.x_shape, ctx.cache, res=_as_bf16_grad(gp), res_up2=1,
                                       res_scale=0.25)
            elif FUSE_GP_ADDS and gp is not None and dz is not None:
                dx = PoolConvBwdDataFn.apply(dz, _as_bf16_grad(gp), W, g, ctx.x_shape, ctx.cache)
            else:
                parts = []
                if dz is not None:
                    parts.append(ConvBwdDataFn.apply(dz, W, g, ctx.x_shape, ctx.cache))
                if gp is not None:
                    parts.append(AvgPool2AdjFn.apply(_as_bf16_grad(gp)))
                dx = parts[0] if len(parts) == 1 else parts[0] + parts[1]
        if dz is not None and _needed(ctx, 1):
            sink = _grad_sink(ctx, 1)
            if sink is not None and sink.is_contiguous(memory_format=CL):
                conv_bwd_weight_raw(x, dz, g, W.shape, out=sink)
            else:
                dW = ConvBwdWeightFn.apply(x, dz, g)
        if dz is not None and ctx.needs_input_grad[2] and _needed(ctx, 2):
            sink = _grad_sink(ctx, 2)
            if sink is not None:
                _sink_chansum(ctx, 2, dz, sink)
            else:
                db = ChanSumFn.apply(dz)
        return dx, dW, db, None, None, None, None, None


# False: the gradient penalty's create_graph backward sums resD's two input
# gradients and ScaleAdd's two output gradients with separate passes (module
# constant for A/B, as FUSE_GP_ACT)
FUSE_GP_ADDS = True


class PoolConvBwdDataFn(torch.autograd.Function):
    """PoolConvFn's dx under create_graph (the gradient penalty's first
    backward): conv^T(dz) + avg_pool2d adjoint(gp) in one data-gradient launch
    (the pooled branch's gradient added in the epilogue, as in the first-order
    path), differentiable: its backward is ConvBwdDataFn's and AvgPool2AdjFn's."""

    @staticmethod
    def forward(ctx, dz, gp, W, g, x_shape, cache):
        ctx.g, ctx.cache = g, cache
        ctx.save_for_backward(dz, W)
        return conv_bwd_data_raw(dz, W, g, x_shape, cache, res=gp, res_up2=1, res_scale=0.25)

    @staticmethod
    def backward(ctx, gdx):
        dz, W = ctx.saved_tensors
        gdx = _as_bf16_grad(gdx)
        g_dz = g_gp = g_W = None
        if ctx.needs_input_grad[0]:
            g_dz = Conv2dFn.apply(gdx, W, None, ctx.g, 0, 0.0, False, ctx.cache)
        if ctx.needs_input_grad[1]:
            g_gp = AvgPool2Fn.apply(gdx)
        if ctx.needs_input_grad[2] and _needed(ctx, 2) and not _sink_wgrad(ctx, 2, gdx, dz, ctx.g, W.shape):
            g_W = ConvBwdWeightFn.apply(gdx, dz, ctx.g)
        return g_dz, g_gp, g_W, None, None, None


class GatedConvBwdDataFn(torch.autograd.Function):
    """Conv2dFn's dx under create_graph when its input x = act(z) came from a
    layer with defer_act=True: conv^T(dz) * act'(x) in one data-gradient launch
    (the producer's ActBwdFn folded in, as in the first-order path).  act' is
    piecewise constant, so x gets no gradient; the double backward masks the
    incoming gradient once and runs ConvBwdDataFn's adjoints on it."""

    @staticmethod
    def forward(ctx, dz, W, x, g, x_shape, cache, act, slope):
        ctx.g, ctx.cache, ctx.act, ctx.slope = g, cache, act, slope
        ctx.save_for_backward(dz, W, x)
        return conv_bwd_data_raw(dz, W, g, x_shape, cache, gate=x, gate_act=act, gate_slope=slope)

    @staticmethod
    def backward(ctx, gdx):
        dz, W, x = ctx.saved_tensors
        gm = ActBwdFn.apply(_as_bf16_grad(gdx), x, ctx.act, ctx.slope)
        g_dz = g_W = None
        if ctx.needs_input_grad[0]:
            g_dz = Conv2dFn.apply(gm, W, None, ctx.g, 0, 0.0, False, ctx.cache)
        if ctx.needs_input_grad[1] and _needed(ctx, 1) and not _sink_wgrad(ctx, 1, gm, dz, ctx.g, W.shape):
            g_W = ConvBwdWeightFn.apply(gm, dz, ctx.g)
        return g_dz, g_W, None, None, None, None, None, None


class ConvBwdDataFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, dz, W, g, x_shape, cache):
        ctx.g, ctx.cache, ctx.x_shape = g, cache, x_shape
        ctx.save_for_backward(dz, W)
        return conv_bwd_data_raw(dz, W, g, x_shape, cache)

    @staticmethod
    def backward(ctx, gdx):
        dz, W = ctx.saved_tensors
        gdx = _as_bf16_grad(gdx)
        g_dz = g_W = None
        if ctx.needs_input_grad[0]:
            g_dz = Conv2dFn.apply(gdx, W, None, ctx.g, 0, 0.0, False, ctx.cache)
        # the gradient penalty's second backward: dW straight into p.grad when it can
        if ctx.needs_input_grad[1] and _needed(ctx, 1) and not _sink_wgrad(ctx, 1, gdx, dz, ctx.g, W.shape):
            g_W = ConvBwdWeightFn.apply(gdx, dz, ctx.g)
        return g_dz, g_W, None, None, None


class ConvBwdWeightFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, dz, g):
        ctx.g = g
        ctx.x_shape = tuple(x.shape)
        ctx.save_for_backward(x, dz)
        K = g.K
        return conv_bwd_weight_raw(x, dz, g, (K, x.shape[1], g.R, g.S))

    @staticmethod
    def backward(ctx, gW):
        x, dz = ctx.saved_tensors
        gx = gdz = None
        if ctx.needs_input_grad[0]:
            gx = ConvBwdDataFn.apply(dz, gW, ctx.g, ctx.x_shape, None)
        if ctx.needs_input_grad[1]:
            gdz = Conv2dFn.apply(x, gW, None, ctx.g, 0, 0.0, False, None)
        return gx, gdz, None


def _mask_src(t, act):
    """The activation tensor an act' mask is read from, as a first-backward
    Function's input: detached when act' is piecewise constant (relu / leaky
    relu -- no gradient flows into it), so the gradient penalty's second
    backward has no edge back into the forward graph.  Attached, autograd ran
    every forward conv's backward there on zero-filled gradients (custom
    Functions materialise the missing ones): a data and a weight gradient per
    conv of the discriminator, all adding zeros (tools/gp_trace.py)."""
    if not DETACH_MASK_SRC:
        return t
    return t.detach() if t is not None and act in (0, ACT_CODES['relu'], ACT_CODES['lrelu']) else t


# On inside Trainer.MA_gradient_penalty's first backward (detached_mask_sources), where
# every parameter's gradient lives in a FlatAdam buffer zeroed before the backward, so a
# bias the second backward no longer reaches keeps its exact-zero gradient as in the
# reference.  Off elsewhere: under the reference's own train.py (torch Adam, zero_grad
# to None) such a bias would get no .grad and Adam would skip its moment update.
# tools/ab_inproc.py "py:eegan_hip.functional.GP_DETACH_MASKS=False" A/Bs the trainer's use.
DETACH_MASK_SRC = False
GP_DETACH_MASKS = True


@contextlib.contextmanager
def detached_mask_sources(on=True):
    global DETACH_MASK_SRC
    prev = DETACH_MASK_SRC
    DETACH_MASK_SRC = bool(on)
    try:
        yield
    finally:
        DETACH_MASK_SRC = prev


class ActBwdFn(torch.autograd.Function):
    """dz = g * act'(y); linear in g (relu/lrelu derivative is piecewise constant)."""

    @staticmethod
    def forward(ctx, g, y, act, slope):
        ctx.act, ctx.slope = act, slope
        ctx.save_for_backward(y)
        return act_bwd_raw(g, y, act, slope)

    @staticmethod
    def backward(ctx, gg):
        (y,) = ctx.saved_tensors
        if ctx.act not in (ACT_CODES['relu'], ACT_CODES['lrelu'], 0) and ctx.needs_input_grad[1]:
            raise NotImplementedError('second derivative through tanh/sigmoid is not used by the step')
        return ActBwdFn.apply(_as_bf16_grad(gg), y, ctx.act, ctx.slope), None, None, None


class ChanSumFn(torch.autograd.Function):
    """bias gradient: per-channel sum over pixels (fp32 [C])."""

    @staticmethod
    def forward(ctx, dz):
        ctx.shape = tuple(dz.shape)
        return chansum_raw(dz)

    @staticmethod
    def backward(ctx, gb):
        N, C, H, W = ctx.shape
        out = empty_nhwc(N, C, H, W, gb.device)
        out.copy_(gb.view(1, C, 1, 1).expand(N, C, H, W))  # broadcast (never on the step's hot path)
        return out


class CastF32Bf16Fn(torch.autograd.Function):
    """fp32 (N,C,H,W) NHWC-dense -> bf16 NHWC (used on grads of fp32-output convs)."""

    @staticmethod
    def forward(ctx, x):
        N, C, H, W = x.shape
        xc = x if (T.is_nhwc(x) and ld_of(x) == C) else x.contiguous(memory_format=torch.channels_last)
        out = empty_nhwc(N, C, H, W, x.device)
        ops.convert(xc.data_ptr(), N * H * W, C, out.data_ptr(), 0, ld_of(out), stream())
        return out

    @staticmethod
    def backward(ctx, g):
        return CastBf16F32Fn.apply(_as_bf16_grad(g))


class CastBf16F32Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        N, C, H, W = x.shape
        out = torch.empty((N, H, W, C), dtype=F32, device=x.device)
        ops.nhwc_to_nchw(x.data_ptr(), ld_of(x), N * H * W, C, 1, out.data_ptr(), stream())
        return out.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, g):
        return CastF32Bf16Fn.apply(g)


class ImageToNhwcFn(torch.autograd.Function):
    """fp32 NCHW image (reference data layout) -> bf16 NHWC; grads return fp32 NCHW."""

    @staticmethod
    def forward(ctx, x):
        return to_nhwc_bf16(x.contiguous())

    @staticmethod
    def backward(ctx, g):
        return ImageToNchwFn.apply(_as_bf16_grad(g))


class ImageToNchwFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        N, C, H, W = x.shape
        out = torch.empty((N, C, H, W), dtype=F32, device=x.device)
        ops.nhwc_to_nchw(x.data_ptr(), ld_of(x), N, C, H * W, out.data_ptr(), stream())
        return out

    @staticmethod
    def backward(ctx, g):
        return ImageToNhwcFn.apply(g)


# ===================================================== pool / combine =====
class AvgPool2Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = to_nhwc_bf16(x)
        N, C, H, W = x.shape
        y = empty_nhwc(N, C, H // 2, W // 2, x.device)
        ops.avgpool2(x.data_ptr(), N, H, W, C, ld_of(x), y.data_ptr(), ld_of(y), stream())
        return y

    @staticmethod
    def backward(ctx, g):
        return AvgPool2AdjFn.apply(_as_bf16_grad(g))


class AvgPool2AdjFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, g):
        N, C, H, W = g.shape
        dx = empty_nhwc(N, C, H * 2, W * 2, g.device)
        ops.upsample2(g.data_ptr(), N, H, W, C, ld_of(g), 0.25, dx.data_ptr(), ld_of(dx), stream())
        return dx

    @staticmethod
    def backward(ctx, gg):
        return AvgPool2Fn.apply(_as_bf16_grad(gg))


class StreamHandoffFn(torch.autograd.Function):
    """Identity at a point where a tensor made on one stream is read on the
    current one (the generator's branch lane, models.Gen.forward_branched).
    Its backward runs on the current (reading) stream and produces the
    gradient that the OTHER stream's backward consumes: the gradient is
    recorded on that stream, so the caching allocator does not hand its memory
    to this stream's next allocation before the other stream's queued reads
    ran (autograd orders the streams, it does not guard the memory)."""

    @staticmethod
    def forward(ctx, x, other):
        ctx.other = other
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        if g is not None and g.is_cuda:
            g.record_stream(ctx.other)
        return g, None


class Upsample2Fn(torch.autograd.Function):
    """F.interpolate(x, scale_factor=2) (nearest); adjoint = 2x2 sum-pool."""

    @staticmethod
    def forward(ctx, x):
        x = to_nhwc_bf16(x)
        N, C, H, W = x.shape
        y = empty_nhwc(N, C, H * 2, W * 2, x.device)
        ops.upsample2(x.data_ptr(), N, H, W, C, ld_of(x), 1.0, y.data_ptr(), ld_of(y), stream())
        return y

    @staticmethod
    def backward(ctx, g):
        g = _as_bf16_grad(g)
        N, C, H, W = g.shape
        dx = empty_nhwc(N, C, H // 2, W // 2, g.device)
        ops.sumpool2(g.data_ptr(), N, H, W, C, ld_of(g), dx.data_ptr(), ld_of(dx), stream())
        return dx


def _scale_raw(x, gamma, alpha=1.0):
    N, C, H, W = x.shape
    out = empty_nhwc(N, C, H, W, x.device)
    ops.scale_add(0, 0, x.data_ptr(), ld_of(x), ptr(gamma), alpha, N * H * W, C, out.data_ptr(), ld_of(out), stream())
    return out


def _dot_raw(x, y):
    N, C, H, W = x.shape
    out = torch.empty(1, dtype=F32, device=x.device)
    ws = workspace(ops.dot_workspace(), x.device)
    ops.dot(x.data_ptr(), ld_of(x), ptr(y), ld_of(y) if y is not None else 0, N * H * W, C, 1.0, ws.data_ptr(),
            out.data_ptr(), 0, stream())
    return out


class ScaleAddFn(torch.autograd.Function):
    """out = res + gamma * h   (gamma: fp32 (1,) parameter; models.py:122,142,278)."""

    @staticmethod
    def forward(ctx, res, h, gamma, h_act=0, h_slope=0.2):
        """h_act: activation that produced h in a layer called with defer_act=True
        (first-order backward folds its derivative into gamma * g; see Conv2dFn)."""
        res = to_nhwc_bf16(res)
        h = to_nhwc_bf16(h)
        N, C, H, W = h.shape
        out = empty_nhwc(N, C, H, W, h.device)
        ops.scale_add(res.data_ptr(), ld_of(res), h.data_ptr(), ld_of(h), gamma.data_ptr(), 1.0, N * H * W, C,
                      out.data_ptr(), ld_of(out), stream())
        ctx.save_for_backward(h, gamma)
        ctx.h_act, ctx.h_slope = h_act, h_slope
        return out

    @staticmethod
    def backward(ctx, g):
        h, gamma = ctx.saved_tensors
        g = _as_bf16_grad(g)
        d_res = g if ctx.needs_input_grad[0] else None
        h_act = ctx.h_act if FUSE_ACT_BWD else 0
        if not torch.is_grad_enabled() and _needed(ctx, 1) and (_needed(ctx, 2) or h_act):
            # first-order: gamma * g [* act'(h)] and <g, h> in one pass, the gain's
            # gradient accumulated straight into gamma.grad when that is the sink
            N, C, H, W = g.shape
            d_h = empty_nhwc(N, C, H, W, g.device)
            sink = _grad_sink(ctx, 2) if _needed(ctx, 2) else None
            d_g = None
            if sink is None:
                d_g = torch.empty(1, dtype=F32, device=g.device)
            ws = workspace(ops.dot_workspace(), g.device)
            ops.scale_dot(g.data_ptr(), ld_of(g), h.data_ptr(), ld_of(h), gamma.data_ptr(), 1.0, N * H * W, C,
                          d_h.data_ptr(), ld_of(d_h), ws.data_ptr(), (sink if d_g is None else d_g).data_ptr(),
                          int(d_g is None), h_act, ctx.h_slope, stream())
            if not _needed(ctx, 2):
                d_g = None
            return d_res, d_h, d_g, None, None
        if FUSE_GP_GATE and FUSE_GP_ACT and h_act and d_res is not None and ctx.needs_input_grad[1]:
            # create_graph with the residual branch's activation deferred here (its
            # producer, resD's conv_r[2], skips its ActBwdFn: _act_deferred -- the same
            # switches, FUSE_ACT_BWD, FUSE_GP_ACT and FUSE_GP_GATE, decide both sides)
            d_res, d_h = ScaleAddGateBwdFn.apply(g, _mask_src(h, h_act), gamma, h_act, ctx.h_slope)
        elif FUSE_GP_ADDS and d_res is not None and ctx.needs_input_grad[1]:
            d_res, d_h = ScaleAddBwdFn.apply(g, gamma)
        else:
            d_h = ScaleFn.apply(g, gamma) if ctx.needs_input_grad[1] else None
        d_g = DotFn.apply(g, h) if _needed(ctx, 2) else None
        return d_res, d_h, d_g, None, None


# False: under create_graph ScaleAddFn does not gate, and resD's conv_r[2] runs its
# activation backward as its own ActBwdFn pass in the gradient penalty's first
# backward (and that pass's backward in the second); module constant for A/B
FUSE_GP_GATE = True


class ScaleAddGateBwdFn(torch.autograd.Function):
    """(g, gamma * g * act'(h)): ScaleAddFn's gradients of (res, z) under
    create_graph, z the pre-activation of the residual branch h = act(z)
    (resD, models.py:270-278: the last LeakyReLU's backward folded in, as the
    first-order path does) -- ONE pass instead of ScaleAddBwdFn's scale and
    conv_r[2]'s ActBwdFn.  act' is piecewise constant, so h gets no gradient.
    The double backward is one pass too: gg_res + gamma * act'(h) * gg_z and
    gamma's <act'(h) * gg_z, g> (eegan_scale_gate), where the composition it
    replaces ran ScaleAddBwdFn's pass and ActBwdFn's backward."""

    @staticmethod
    def forward(ctx, g, h, gamma, act, slope):
        ctx.act, ctx.slope = act, slope
        ctx.save_for_backward(g, h, gamma)
        N, C, H, W = g.shape
        out = empty_nhwc(N, C, H, W, g.device)
        ops.scale_gate(g.data_ptr(), ld_of(g), h.data_ptr(), ld_of(h), act, slope, gamma.data_ptr(), 1.0, N * H * W, C,
                       None, 0, None, 0, out.data_ptr(), ld_of(out), None, None, 0, stream())
        return g, out

    @staticmethod
    def backward(ctx, gg_res, gg_z):
        g, h, gamma = ctx.saved_tensors
        if gg_z is None:
            return gg_res, None, None, None, None
        gg_z = _as_bf16_grad(gg_z)
        if gg_res is not None:
            gg_res = _as_bf16_grad(gg_res)
        need_gamma = _needed(ctx, 2)
        if torch.is_grad_enabled():   # a third-order pass: composed of differentiable Functions
            m = ActBwdFn.apply(gg_z, h.detach(), ctx.act, ctx.slope)
            out = ScaleFn.apply(m, gamma)
            if gg_res is not None:
                out = out + gg_res
            return out, None, (DotFn.apply(m, g) if need_gamma else None), None, None
        N, C, H, W = gg_z.shape
        out = empty_nhwc(N, C, H, W, gg_z.device)
        d_g = sink = ws = None
        if need_gamma:
            sink = _grad_sink(ctx, 2)
            d_g = torch.empty(1, dtype=F32, device=g.device) if sink is None else None
            ws = workspace(ops.dot_workspace(), g.device)
        ops.scale_gate(gg_z.data_ptr(), ld_of(gg_z), h.data_ptr(), ld_of(h), ctx.act, ctx.slope, gamma.data_ptr(), 1.0,
                       N * H * W, C, ptr(gg_res), ld_of(gg_res) if gg_res is not None else 0,
                       g.data_ptr() if need_gamma else None, ld_of(g) if need_gamma else 0, out.data_ptr(),
                       ld_of(out), ptr(ws), (sink if d_g is None else d_g).data_ptr() if need_gamma else None,
                       int(need_gamma and d_g is None), stream())
        return out, None, d_g, None, None


class ScaleAddBwdFn(torch.autograd.Function):
    """(g, gamma * g): ScaleAddFn's gradients of (res, h) under create_graph as
    ONE node, so the double backward sums the two paths' gradients, scales one
    and takes gamma's <gg_h, g> in a single pass (eegan_scale_dot_res) instead
    of ScaleFn's backward, DotFn and autograd's add.  The first output is g
    itself (autograd returns it as a view attached to this node)."""

    @staticmethod
    def forward(ctx, g, gamma):
        ctx.save_for_backward(g, gamma)
        return g, _scale_raw(g, gamma)

    @staticmethod
    def backward(ctx, gg_res, gg_h):
        g, gamma = ctx.saved_tensors
        if gg_h is None:
            return gg_res, None
        gg_h = _as_bf16_grad(gg_h)
        if gg_res is not None:
            gg_res = _as_bf16_grad(gg_res)
        need_gamma = _needed(ctx, 1)
        if torch.is_grad_enabled():   # a third-order pass: composed of differentiable Functions
            out = ScaleFn.apply(gg_h, gamma)
            if gg_res is not None:
                out = out + gg_res
            return out, (DotFn.apply(gg_h, g) if need_gamma else None)
        N, C, H, W = gg_h.shape
        out = empty_nhwc(N, C, H, W, gg_h.device)
        if not need_gamma:
            ops.scale_add(ptr(gg_res), ld_of(gg_res) if gg_res is not None else 0, gg_h.data_ptr(), ld_of(gg_h),
                          gamma.data_ptr(), 1.0, N * H * W, C, out.data_ptr(), ld_of(out), stream())
            return out, None
        sink = _grad_sink(ctx, 1)
        d_g = torch.empty(1, dtype=F32, device=g.device) if sink is None else None
        ws = workspace(ops.dot_workspace(), g.device)
        ops.scale_dot_res(gg_h.data_ptr(), ld_of(gg_h), g.data_ptr(), ld_of(g), gamma.data_ptr(), 1.0, N * H * W, C,
                          ptr(gg_res), ld_of(gg_res) if gg_res is not None else 0, out.data_ptr(), ld_of(out),
                          ws.data_ptr(), (sink if d_g is None else d_g).data_ptr(), int(d_g is None), stream())
        return out, d_g


class ScaleFn(torch.autograd.Function):
    """gamma * x with gamma a device scalar."""

    @staticmethod
    def forward(ctx, x, gamma):
        ctx.save_for_backward(x, gamma)
        return _scale_raw(x, gamma)

    @staticmethod
    def backward(ctx, g):
        x, gamma = ctx.saved_tensors
        g = _as_bf16_grad(g)
        gx = ScaleFn.apply(g, gamma) if ctx.needs_input_grad[0] else None
        gg = DotFn.apply(g, x) if ctx.needs_input_grad[1] else None
        return gx, gg


class DotFn(torch.autograd.Function):
    """<x, y> summed over all elements -> fp32 (1,)."""

    @staticmethod
    def forward(ctx, x, y):
        ctx.save_for_backward(x, y)
        return _dot_raw(x, y)

    @staticmethod
    def backward(ctx, gs):
        x, y = ctx.saved_tensors
        gs = gs.reshape(1).contiguous()
        gx = ScaleFn.apply(y, gs) if ctx.needs_input_grad[0] else None
        gy = ScaleFn.apply(x, gs) if ctx.needs_input_grad[1] else None
        return gx, gy


class BatchCatFn(torch.autograd.Function):
    """torch.cat(parts, 0) for NHWC bf16 activations (same C, H, W): one copy
    per part into a fresh NHWC buffer; the backward returns views of the
    gradient (differentiable slicing)."""

    @staticmethod
    def forward(ctx, *parts):
        parts = [to_nhwc_bf16(p) for p in parts]
        N0, C, H, W = parts[0].shape
        ns = [p.shape[0] for p in parts]
        out = empty_nhwc(sum(ns), C, H, W, parts[0].device)
        o = 0
        for p, n in zip(parts, ns):
            out[o:o + n].copy_(p)
            o += n
        ctx.ns = ns
        return out

    @staticmethod
    def backward(ctx, g):
        outs, o = [], 0
        for n in ctx.ns:
            outs.append(g[o:o + n])
            o += n
        return tuple(outs)


class CatTileFn(torch.autograd.Function):
    """torch.cat((feat, cond.view(-1,E,1,1).repeat(1,1,H,W)), 1) (models.py:302-304, 327-331)."""

    @staticmethod
    def forward(ctx, feat, cond):
        feat = to_nhwc_bf16(feat)
        cond = cond.reshape(cond.shape[0], -1).float().contiguous()
        N, C, H, W = feat.shape
        E = cond.shape[1]
        out = empty_nhwc(N, C + E, H, W, feat.device)
        ops.cat_tile(feat.data_ptr(), ld_of(feat), cond.data_ptr(), N, H * W, C, E, out.data_ptr(), ld_of(out),
                     stream())
        ctx.dims = (N, C, H, W, E)
        return out

    @staticmethod
    def backward(ctx, g):
        return CatTileBwdFn.apply(_as_bf16_grad(g), ctx.dims)


class CatTileBwdFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, g, dims):
        N, C, H, W, E = dims
        ctx.dims = dims
        df = empty_nhwc(N, C, H, W, g.device)
        dc = torch.empty((N, E), dtype=F32, device=g.device)
        ops.cat_tile_bwd(g.data_ptr(), ld_of(g), N, H * W, C, E, df.data_ptr(), ld_of(df), dc.data_ptr(), stream())
        return df, dc

    @staticmethod
    def backward(ctx, gf, gc):
        N, C, H, W, E = ctx.dims
        if gf is None:
            gf = torch.zeros_like(empty_nhwc(N, C, H, W, gc.device))
        if gc is None:
            gc = torch.zeros((N, E), dtype=F32, device=gf.device)
        return CatTileFn.apply(_as_bf16_grad(gf), gc), None


class CatChannelsFn(torch.autograd.Function):
    """torch.cat(parts, 1) for NHWC activations (Inception branch concat).  The
    backward hands each branch a strided view of the incoming gradient (no copy)."""

    @staticmethod
    def forward(ctx, *parts):
        parts = [to_nhwc_bf16(p) for p in parts]
        N, _, H, W = parts[0].shape
        Cs = [p.shape[1] for p in parts]
        out = empty_nhwc(N, sum(Cs), H, W, parts[0].device)
        ldo = ld_of(out)
        if len(parts) <= 8 and all(c % 8 == 0 and ld_of(p) % 8 == 0 for p, c in zip(parts, Cs)):
            n = len(parts)
            ptrs = (ctypes.c_void_p * n)(*[p.data_ptr() for p in parts])
            lds = (ctypes.c_int * n)(*[ld_of(p) for p in parts])
            cs = (ctypes.c_int * n)(*Cs)
            ops.cat_channels(ptrs, lds, cs, n, N * H * W, out.data_ptr(), ldo, stream())
        else:
            off = 0
            for p, c in zip(parts, Cs):
                ops.scale_add(0, 0, p.data_ptr(), ld_of(p), 0, 1.0, N * H * W, c, out[:, off:off + c].data_ptr(),
                              ldo, stream())
                off += c
        ctx.Cs = Cs
        return out

    @staticmethod
    def backward(ctx, g):
        g = _as_bf16_grad(g)
        outs, off = [], 0
        for c in ctx.Cs:
            outs.append(g[:, off:off + c])
            off += c
        return tuple(outs)


class SplitChannelsFn(torch.autograd.Function):
    """Channel-slice views y[:, o_i : o_i + C_i] of one NHWC activation (the
    outputs of stacked 1x1 convs); backward assembles the slices' gradients
    into one buffer in one launch (eegan_cat_channels) instead of autograd's
    zero-filled slice gradients and adds."""

    @staticmethod
    def forward(ctx, y, sizes):
        outs, o = [], 0
        for c in sizes:
            outs.append(y[:, o:o + c])
            o += c
        ctx.sizes = tuple(sizes)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gs):
        parts = []
        for g, c in zip(gs, ctx.sizes):
            if g is None:
                ref = next(x for x in gs if x is not None)
                N, _, H, W = ref.shape
                g = empty_nhwc(N, c, H, W, ref.device)
                g.zero_()
            parts.append(_as_bf16_grad(g))
        return CatChannelsFn.apply(*parts), None


# ================================================================ linear ===
def _gemm(tag, A, sai, sak, B, sbk, sbj, C, ldc, M, N, K, bias, act, alpha, beta):
    _launch('gemm_f32', 2.0 * M * N * K, 4.0 * (M * K + K * N + M * N), lambda: ops.gemm_f32(
        A, sai, sak, B, sbk, sbj, C, ldc, M, N, K, bias, act, alpha, beta, stream()),
        key='%s M%d N%d K%d' % (tag, M, N, K) if TIMER is not None else None)


class LinearFn(torch.autograd.Function):
    """y = act(x W^T + b), fp32 (first order)."""

    @staticmethod
    def forward(ctx, x, W, b, act):
        x2 = x.reshape(-1, x.shape[-1]).float().contiguous()
        M, K = x2.shape
        N = W.shape[0]
        y = torch.empty((M, N), dtype=F32, device=x.device)
        _gemm('linear_fwd', x2.data_ptr(), K, 1, W.data_ptr(), 1, K, y.data_ptr(), N, M, N, K, ptr(b), act, 1.0, 0.0)
        ctx.act = act
        ctx.in_shape = tuple(x.shape)
        ctx.save_for_backward(x2, W, y if act else None)
        return y.reshape(*x.shape[:-1], N)

    @staticmethod
    def backward(ctx, gy):
        x2, W, y = ctx.saved_tensors
        M, K = x2.shape
        N = W.shape[0]
        g = gy.reshape(M, N).float().contiguous()
        if ctx.act:
            dz = torch.empty_like(g)
            ops.act_bwd_f32(g.data_ptr(), y.data_ptr(), M * N, ctx.act, 0.2, dz.data_ptr(), stream())
            g = dz
        dx = dW = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty((M, K), dtype=F32, device=g.device)
            _gemm('linear_dx', g.data_ptr(), N, 1, W.data_ptr(), K, 1, dx.data_ptr(), K, M, K, N, 0, 0, 1.0, 0.0)
            dx = dx.reshape(ctx.in_shape)
        if _needed(ctx, 1):
            sink = _grad_sink(ctx, 1)
            dst = sink if sink is not None else torch.empty((N, K), dtype=F32, device=g.device)
            _gemm('linear_dw', g.data_ptr(), 1, N, x2.data_ptr(), K, 1, dst.data_ptr(), K, N, K, M, 0, 0, 1.0,
                  1.0 if sink is not None else 0.0)
            dW = dst if sink is None else None
        if ctx.needs_input_grad[2] and _needed(ctx, 2):
            sink = _grad_sink(ctx, 2)
            dst = sink if sink is not None else torch.empty(N, dtype=F32, device=g.device)
            ops.colsum_f32(g.data_ptr(), N, M, N, dst.data_ptr(), int(sink is not None), stream())
            db = dst if sink is None else None
        return dx, dW, db, None


# ================================================= grouped affine MLPs ===
# EEGAN_GROUPED_MLP=0 runs every affine_ssa MLP as its own LinearFn pair.
GROUPED_MLP = os.environ.get('EEGAN_GROUPED_MLP', '1') != '0'
_ONES = {}


def _ones(n, dev):
    key = (dev, n)
    if key not in _ONES:
        _ONES[key] = torch.ones(n, dtype=F32, device=dev)
    return _ONES[key]


def _gemm_grouped(tag, descs):
    if not descs:
        return
    arr = (GemmDesc * len(descs))(*[GemmDesc(*d) for d in descs])
    flops = sum(2.0 * d[11] * d[12] * d[13] for d in descs)
    nbytes = sum(4.0 * (d[11] * d[13] + d[13] * d[12] + d[11] * d[12]) for d in descs)
    _launch('gemm_f32', flops, nbytes, lambda: ops.gemm_f32_grouped(arr, len(descs), stream()),
            key='%s x%d' % (tag, len(descs)) if TIMER is not None else None)


def _gd(A, sai, sak, B, sbk, sbj, C, ldc, M, N, K, bias=0, act=0, beta=0.0, gate=0, ldg=0, gate_act=0):
    """GemmDesc field order: A, B, C, bias, gate, sai, sak, sbk, sbj, ldc, ldg, M, N, K, act, gate_act, alpha, beta."""
    return (A, B, C, bias, gate, sai, sak, sbk, sbj, ldc, ldg, M, N, K, act, gate_act, 1.0, beta)


class AffineMLPsFn(torch.autograd.Function):
    """Every affine_ssa fc_gamma / fc_beta MLP of one generator pass
    (Linear -> ReLU -> Linear, models.py:51-60) as grouped GEMMs: 2 forward
    launches and 6 backward launches (+ one sum per conditioning input)
    instead of ~7 small launches per MLP.  Same products in the same order
    as LinearFn, so the outputs and gradients are bit-identical to it.

    apply(*conds, *params, cidx, nconds): cidx[g] picks MLP g's input among
    conds; params = (W1, b1, W2, b2) per MLP.  Returns one (B, N_g) output per
    MLP.  (The non-tensor arguments come last: ctx.next_functions only lists
    the leading inputs, so tensor positions must match needs_input_grad.)"""

    @staticmethod
    def forward(ctx, *args):
        cidx, nconds = args[-2], args[-1]
        args = args[:-2]
        conds = [x.reshape(x.shape[0], -1).float().contiguous() for x in args[:nconds]]
        params = args[nconds:]
        G = len(params) // 4
        Bn, K = conds[0].shape
        Hd = params[0].shape[0]
        dev = conds[0].device
        H = torch.empty((G, Bn, Hd), dtype=F32, device=dev)
        ys = []
        d1, d2 = [], []
        for g in range(G):
            W1, b1, W2, b2 = params[4 * g:4 * g + 4]
            N = W2.shape[0]
            y = torch.empty((Bn, N), dtype=F32, device=dev)
            ys.append(y)
            d1.append(_gd(conds[cidx[g]].data_ptr(), K, 1, W1.data_ptr(), 1, K, H[g].data_ptr(), Hd, Bn, Hd, K,
                          bias=ptr(b1), act=ACT_CODES['relu']))
            d2.append(_gd(H[g].data_ptr(), Hd, 1, W2.data_ptr(), 1, Hd, y.data_ptr(), N, Bn, N, Hd, bias=ptr(b2)))
        _gemm_grouped('mlp_fwd1', d1)
        _gemm_grouped('mlp_fwd2', d2)
        ctx.cidx, ctx.nconds, ctx.G = tuple(cidx), nconds, G
        ctx.save_for_backward(H, *conds, *params)
        return tuple(ys)

    @staticmethod
    def backward(ctx, *gys):
        saved = ctx.saved_tensors
        H, conds, params = saved[0], saved[1:1 + ctx.nconds], saved[1 + ctx.nconds:]
        G, Bn, Hd = H.shape
        K = conds[0].shape[1]
        dev = H.device
        ones = _ones(Bn, dev)
        off = ctx.nconds  # needs_input_grad index of params[0]
        grads = [None] * len(params)
        d1, d2 = [], []
        dH = torch.empty_like(H)
        need_c = [ctx.needs_input_grad[i] for i in range(ctx.nconds)]
        DCP = torch.empty((G, Bn, K), dtype=F32, device=dev) if any(need_c) else None
        live = []

        def sink_or_new(i, shape):
            s_ = _grad_sink(ctx, off + i) if _needed(ctx, off + i) else None
            if s_ is not None:
                return s_, 1.0, None
            if not _needed(ctx, off + i):
                return None, 0.0, None
            t = torch.empty(shape, dtype=F32, device=dev)
            return t, 0.0, t

        for g in range(G):
            gy = gys[g]
            if gy is None:
                continue
            live.append(g)
            gy = gy.reshape(Bn, -1).float().contiguous()
            W1, b1, W2, b2 = params[4 * g:4 * g + 4]
            N = W2.shape[0]
            dst, beta, ret = sink_or_new(4 * g + 2, (N, Hd))
            if dst is not None:
                d1.append(_gd(gy.data_ptr(), 1, N, H[g].data_ptr(), Hd, 1, dst.data_ptr(), Hd, N, Hd, Bn, beta=beta))
                grads[4 * g + 2] = ret
            dst, beta, ret = sink_or_new(4 * g + 3, (N,))
            if dst is not None:
                d1.append(_gd(gy.data_ptr(), 1, N, ones.data_ptr(), 1, 0, dst.data_ptr(), 1, N, 1, Bn, beta=beta))
                grads[4 * g + 3] = ret
            d1.append(_gd(gy.data_ptr(), N, 1, W2.data_ptr(), Hd, 1, dH[g].data_ptr(), Hd, Bn, Hd, N,
                          gate=H[g].data_ptr(), ldg=Hd, gate_act=ACT_CODES['relu']))
            dst, beta, ret = sink_or_new(4 * g, (Hd, K))
            if dst is not None:
                d2.append(_gd(dH[g].data_ptr(), 1, Hd, conds[ctx.cidx[g]].data_ptr(), K, 1, dst.data_ptr(), K,
                              Hd, K, Bn, beta=beta))
                grads[4 * g] = ret
            dst, beta, ret = sink_or_new(4 * g + 1, (Hd,))
            if dst is not None:
                d2.append(_gd(dH[g].data_ptr(), 1, Hd, ones.data_ptr(), 1, 0, dst.data_ptr(), 1, Hd, 1, Bn, beta=beta))
                grads[4 * g + 1] = ret
            if need_c[ctx.cidx[g]]:
                d2.append(_gd(dH[g].data_ptr(), Hd, 1, W1.data_ptr(), K, 1, DCP[g].data_ptr(), K, Bn, K, Hd))
        _gemm_grouped('mlp_bwd1', d1)
        _gemm_grouped('mlp_bwd2', d2)
        dconds = [None] * ctx.nconds
        for ci in range(ctx.nconds):
            if not need_c[ci]:
                continue
            gs = [g for g in live if ctx.cidx[g] == ci]
            if not gs:
                continue
            if gs == list(range(gs[0], gs[-1] + 1)):
                dconds[ci] = DCP[gs[0]:gs[-1] + 1].sum(0)
            else:
                dconds[ci] = DCP[gs].sum(0)
        return (*dconds, *grads, None, None)


# =========================================================== SyncBN path ===
def _allreduce_f64(t):
    if SYNC_BN_ALLREDUCE is not None:  # installed by eegan_hip.dist for world > 1 (or a forced rehearsal)
        SYNC_BN_ALLREDUCE(t)


class BnModFn(torch.autograd.Function):
    """SyncBN (training statistics) + affine / affine_ssa modulation + act,
    optionally reading x through a nearest-2x upsample.  mode 0: affine BN
    (w, b may be None); mode 1: (gam*m+1)*xhat + bet*m with gam/bet [N][C]
    and m [N,1,Ho,Wo] fp32."""

    @staticmethod
    def forward(ctx, x, w, b, gam, bet, mask, bn, mode, act, slope, up2):
        x = to_nhwc_bf16(x)
        N, C, H, W = x.shape
        P = N * H * W
        dev = x.device
        s = stream()
        count = float(P * (4 if up2 else 1))
        # statistics (+ cross-rank all-reduce of (sum, sumsq))
        ws = workspace(ops.bn_stats_workspace(P, C), dev)
        sums = torch.empty(2 * C, dtype=torch.float64, device=dev)
        ops.bn_stats(x.data_ptr(), P, C, ld_of(x), ws.data_ptr(), sums.data_ptr(), s)
        world = _syncbn_world()
        if world > 1:
            _allreduce_f64(sums)
            count *= world
        stats = torch.empty(3 * C, dtype=F32, device=dev)
        clamp_mode = 1 if (world > 1 or SYNC_BN_FORCE_MULTI) else 0
        rm = bn.running_mean if (bn is not None and bn.track_running_stats) else None
        rv = bn.running_var if rm is not None else None
        # (the reference calls F.batch_norm directly, so num_batches_tracked never moves)
        Ho, Wo = (H * 2, W * 2) if up2 else (H, W)
        gam_c = gam.float().contiguous() if gam is not None else None
        bet_c = bet.float().contiguous() if bet is not None else None
        mask_c = mask.float().contiguous() if mask is not None else None
        d = BnModDesc(x.data_ptr(), N, H, W, C, ld_of(x), int(up2), stats.data_ptr(), mode, ptr(w), ptr(b),
                      ptr(gam_c), ptr(bet_c), ptr(mask_c), act, slope)
        y = empty_nhwc(N, C, Ho, Wo, dev)
        # finalize (mean / inv_std / running statistics into `stats`) folded into the apply launch
        # (one launch less per BN call; in-process A/B against the separate finalize: 739.6 vs
        # 739.5 img/s -- launch count on the generator's chain is not what bounds it)
        ops.bnmod_fwd_fin(d, sums.data_ptr(), count, 4.0 if up2 else 1.0, bn.eps if bn is not None else 1e-5,
                          bn.momentum if bn is not None else 0.1, clamp_mode, ptr(rm), ptr(rv), y.data_ptr(),
                          ld_of(y), s)
        ctx.meta = (mode, act, slope, up2, count)
        ctx.save_for_backward(x, w, b, gam_c, bet_c, mask_c, stats)
        return y

    @staticmethod
    def backward(ctx, g):
        x, w, b, gam, bet, mask, stats = ctx.saved_tensors
        mode, act, slope, up2, count = ctx.meta
        g = to_nhwc_bf16(g)
        N, C, H, W = x.shape
        dev = x.device
        s = stream()
        d = BnModDesc(x.data_ptr(), N, H, W, C, ld_of(x), int(up2), stats.data_ptr(), mode, ptr(w), ptr(b),
                      ptr(gam), ptr(bet), ptr(mask), act, slope)
        ws = workspace(ops.bnmod_bwd_workspace(d), dev)
        if mode == 0:
            d0 = torch.empty(C, dtype=F32, device=dev)
            d1 = torch.empty(C, dtype=F32, device=dev)
        else:
            d0 = torch.empty((N, C), dtype=F32, device=dev)
            d1 = torch.empty((N, C), dtype=F32, device=dev)
        Ho, Wo = (H * 2, W * 2) if up2 else (H, W)
        dmask = torch.empty((N, 1, Ho, Wo), dtype=F32, device=dev) if (mode == 1 and ctx.needs_input_grad[5]) else None
        chan = torch.empty(2 * C, dtype=torch.float64, device=dev)
        ops.bnmod_bwd(d, g.data_ptr(), ld_of(g), ws.data_ptr(), d0.data_ptr(), d1.data_ptr(), ptr(dmask),
                      chan.data_ptr(), s)
        _allreduce_f64(chan)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = empty_nhwc(N, C, H, W, dev)
            ops.bnmod_bwd_dx(d, g.data_ptr(), ld_of(g), chan.data_ptr(), count, dx.data_ptr(), ld_of(dx), s)
        if mode == 0:
            dw = d0 if (w is not None and ctx.needs_input_grad[1]) else None
            db = d1 if (b is not None and ctx.needs_input_grad[2]) else None
            return dx, dw, db, None, None, None, None, None, None, None, None
        dg = d0 if ctx.needs_input_grad[3] else None
        dbt = d1 if ctx.needs_input_grad[4] else None
        return dx, None, None, dg, dbt, dmask, None, None, None, None, None


class BnEvalFn(torch.autograd.Function):
    """eval-mode BN (running statistics) = per-channel affine + act (sampling only)."""

    @staticmethod
    def forward(ctx, x, scale, shift, act, slope, up2):
        x = to_nhwc_bf16(x)
        N, C, H, W = x.shape
        C_ = scale.numel()
        stats = torch.cat([torch.zeros(C_, device=x.device), torch.ones(C_, device=x.device),
                           torch.ones(C_, device=x.device)]).float()
        d = BnModDesc(x.data_ptr(), N, H, W, C, ld_of(x), int(up2), stats.data_ptr(), 0, scale.data_ptr(),
                      shift.data_ptr(), 0, 0, 0, act, slope)
        Ho, Wo = (H * 2, W * 2) if up2 else (H, W)
        y = empty_nhwc(N, C, Ho, Wo, x.device)
        ops.bnmod_fwd(d, y.data_ptr(), ld_of(y), stream())
        ctx.save_for_backward(y, scale)
        ctx.act, ctx.slope, ctx.up2 = act, slope, up2
        return y

    @staticmethod
    def backward(ctx, g):  # not on the training path (G runs in train mode there)
        y, scale = ctx.saved_tensors
        g = to_nhwc_bf16(g)
        dz = act_bwd_raw(g, y, ctx.act, ctx.slope) if ctx.act else g
        dx = dz.float() * scale.view(1, -1, 1, 1)
        if ctx.up2:
            N, C, H, W = dx.shape
            dx = dx.reshape(N, C, H // 2, 2, W // 2, 2).sum((3, 5))
        return to_nhwc_bf16(dx.contiguous()), None, None, None, None, None


# ================================================================= masks ===
class MaskResizeSigmoidFn(torch.autograd.Function):
    """sigmoid(F.interpolate(m, size, mode='bilinear', align_corners=True)) on
    fp32 [N,1,h,w] masks (models.py:220-221, 231-232)."""

    @staticmethod
    def forward(ctx, m, size):
        m = m.float().contiguous()
        N, Cm, h, w = m.shape
        out = torch.empty((N, Cm, size, size), dtype=F32, device=m.device)
        ops.bilinear(m.data_ptr(), 1, N, h, w, Cm, Cm, size, size, 1, 1, out.data_ptr(), 1, Cm, stream())
        ctx.dims = (N, Cm, h, w, size)
        ctx.save_for_backward(out)
        return out

    @staticmethod
    def backward(ctx, g):
        (out,) = ctx.saved_tensors
        N, Cm, h, w, size = ctx.dims
        g = g.float().contiguous()
        dm = torch.empty((N, Cm, h, w), dtype=F32, device=g.device)
        ops.bilinear_bwd(g.data_ptr(), 1, out.data_ptr(), 1, Cm, N, h, w, Cm, size, size, 1, 1, dm.data_ptr(),
                         stream())
        return dm, None


class BilinearFn(torch.autograd.Function):
    """F.interpolate(x, size, mode='bilinear', align_corners=False) on bf16 NHWC
    (CNN_ENCODER input resize, DAMSM.py:173)."""

    @staticmethod
    def forward(ctx, x, Ho, Wo):
        x = to_nhwc_bf16(x)
        N, C, H, W = x.shape
        y = empty_nhwc(N, C, Ho, Wo, x.device)
        ops.bilinear(x.data_ptr(), 0, N, H, W, C, ld_of(x), Ho, Wo, 0, 0, y.data_ptr(), 0, ld_of(y), stream())
        ctx.dims = (N, C, H, W, Ho, Wo)
        return y

    @staticmethod
    def backward(ctx, g):
        N, C, H, W, Ho, Wo = ctx.dims
        g = to_nhwc_bf16(g)
        d32 = torch.empty((N, H, W, C), dtype=F32, device=g.device)
        ops.bilinear_bwd(g.data_ptr(), 0, 0, 0, ld_of(g), N, H, W, C, Ho, Wo, 0, 0, d32.data_ptr(), stream())
        dx = empty_nhwc(N, C, H, W, g.device)
        ops.convert(d32.data_ptr(), N * H * W, C, dx.data_ptr(), 0, ld_of(dx), stream())
        return dx, None, None


class FcToNhwcFn(torch.autograd.Function):
    """Gen.fc output (N, C*16) fp32 -> view(N, C, 4, 4) as NHWC bf16 (models.py:228-230)."""

    @staticmethod
    def forward(ctx, x, C):
        x = x.float().contiguous()
        N = x.shape[0]
        y = empty_nhwc(N, C, 4, 4, x.device)
        ops.fc_to_nhwc(x.data_ptr(), 1, N, C, 16, y.data_ptr(), ld_of(y), stream())
        ctx.C = C
        return y

    @staticmethod
    def backward(ctx, g):
        g = to_nhwc_bf16(g)
        N = g.shape[0]
        dx = torch.empty((N, ctx.C * 16), dtype=F32, device=g.device)
        ops.nhwc_to_fc(g.data_ptr(), ld_of(g), N, ctx.C, 16, dx.data_ptr(), 1, stream())
        return dx, None


# ============================================================ Inception ====
class MaxPool3s2Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = to_nhwc_bf16(x)
        N, C, H, W = x.shape
        Ho, Wo = (H - 3) // 2 + 1, (W - 3) // 2 + 1
        y = empty_nhwc(N, C, Ho, Wo, x.device)
        arg = torch.empty(N * Ho * Wo * C, dtype=torch.uint8, device=x.device)
        ops.maxpool3s2(x.data_ptr(), N, H, W, C, ld_of(x), y.data_ptr(), ld_of(y), arg.data_ptr(), stream())
        ctx.dims = (N, C, H, W)
        ctx.save_for_backward(arg)
        return y

    @staticmethod
    def backward(ctx, g):
        (arg,) = ctx.saved_tensors
        N, C, H, W = ctx.dims
        g = to_nhwc_bf16(g)
        dx = empty_nhwc(N, C, H, W, g.device)
        ops.maxpool3s2_bwd(g.data_ptr(), ld_of(g), arg.data_ptr(), N, H, W, C, dx.data_ptr(), ld_of(dx), stream())
        return dx


class AvgPool3s1Fn(torch.autograd.Function):
    """avg_pool2d(3, 1, 1, count_include_pad=True): self-adjoint."""

    @staticmethod
    def forward(ctx, x):
        x = to_nhwc_bf16(x)
        N, C, H, W = x.shape
        y = empty_nhwc(N, C, H, W, x.device)
        ops.avgpool3s1(x.data_ptr(), N, H, W, C, ld_of(x), y.data_ptr(), ld_of(y), stream())
        return y

    @staticmethod
    def backward(ctx, g):
        g = to_nhwc_bf16(g)
        N, C, H, W = g.shape
        dx = empty_nhwc(N, C, H, W, g.device)
        ops.avgpool3s1(g.data_ptr(), N, H, W, C, ld_of(g), dx.data_ptr(), ld_of(dx), stream())
        return dx


class GlobalAvgPoolFn(torch.autograd.Function):
    """mean over H*W -> fp32 (N, C)."""

    @staticmethod
    def forward(ctx, x):
        x = to_nhwc_bf16(x)
        N, C, H, W = x.shape
        y = torch.empty((N, C), dtype=F32, device=x.device)
        ops.global_avgpool(x.data_ptr(), ld_of(x), N, H * W, C, y.data_ptr(), 1, stream())
        ctx.dims = (N, C, H, W)
        return y

    @staticmethod
    def backward(ctx, g):
        N, C, H, W = ctx.dims
        g = g.float().contiguous()
        dx = empty_nhwc(N, C, H, W, g.device)
        ops.global_avgpool_bwd(g.data_ptr(), 1, N, H * W, C, dx.data_ptr(), ld_of(dx), stream())
        return dx


# ================================================================ losses ===
class DoutReduceFn(torch.autograd.Function):
    """mode 0 mean(relu(1-x)), 1 mean(relu(1+x)), 2 -mean(x), 3 mean(x) (train.py:342-417)."""

    @staticmethod
    def forward(ctx, x, mode):
        xc = x.float().contiguous()
        out = torch.empty((), dtype=F32, device=x.device)
        ops.dout_reduce(xc.data_ptr(), xc.numel(), mode, out.data_ptr(), stream())
        ctx.mode = mode
        ctx.shape = x.shape
        ctx.save_for_backward(xc)
        return out

    @staticmethod
    def backward(ctx, g):
        (xc,) = ctx.saved_tensors
        g = g.float().reshape(1).contiguous()
        dx = torch.empty_like(xc)
        ops.dout_reduce_bwd(xc.data_ptr(), xc.numel(), ctx.mode, g.data_ptr(), dx.data_ptr(), stream())
        return dx.reshape(ctx.shape), None


class DoutReduce3Fn(torch.autograd.Function):
    """The three D-loss reductions of a batched head output x = [real; mismatch;
    fake] (Trainer._d_heads_batched): DoutReduceFn on x[0:B] (mode m0),
    x[2B:3B] (m1), x[B:2B] (m2) -- one gradient buffer for x instead of a
    zero-filled buffer, a copy and an add per slice."""

    @staticmethod
    def forward(ctx, x, B, modes):
        xc = x.float().contiguous()
        per = xc.numel() // 3
        outs = [torch.empty((), dtype=F32, device=x.device) for _ in range(3)]
        for o, sl, m in zip(outs, (0, 2, 1), modes):
            ops.dout_reduce(xc.data_ptr() + 4 * sl * per, per, m, o.data_ptr(), stream())
        ctx.modes, ctx.shape = modes, x.shape
        ctx.save_for_backward(xc)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gs):
        (xc,) = ctx.saved_tensors
        per = xc.numel() // 3
        dx = torch.empty_like(xc)
        for g, sl, m in zip(gs, (0, 2, 1), ctx.modes):
            g = torch.zeros(1, dtype=F32, device=xc.device) if g is None else g.float().reshape(1).contiguous()
            ops.dout_reduce_bwd(xc.data_ptr() + 4 * sl * per, per, m, g.data_ptr(), dx.data_ptr() + 4 * sl * per,
                                stream())
        return dx.reshape(ctx.shape), None, None


class BceLogits3Fn(torch.autograd.Function):
    """BceLogitsFn(x[0:B], t), (x[2B:3B], t), (x[B:2B], t) of a batched class
    head output, with one gradient buffer (see DoutReduce3Fn)."""

    @staticmethod
    def forward(ctx, x, target):
        xc = x.float().contiguous()
        tc = target.float().contiguous()
        per = xc.numel() // 3
        outs = [torch.empty((), dtype=F32, device=x.device) for _ in range(3)]
        for o, sl in zip(outs, (0, 2, 1)):
            ops.bce_logits(xc.data_ptr() + 4 * sl * per, tc.data_ptr(), per, o.data_ptr(), stream())
        ctx.shape = x.shape
        ctx.save_for_backward(xc, tc)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gs):
        xc, tc = ctx.saved_tensors
        per = xc.numel() // 3
        dx = torch.empty_like(xc)
        for g, sl in zip(gs, (0, 2, 1)):
            g = torch.zeros(1, dtype=F32, device=xc.device) if g is None else g.float().reshape(1).contiguous()
            ops.bce_logits_bwd(xc.data_ptr() + 4 * sl * per, tc.data_ptr(), per, g.data_ptr(),
                               dx.data_ptr() + 4 * sl * per, stream())
        return dx.reshape(ctx.shape), None


class HeadsGatherFn(torch.autograd.Function):
    """[f[:B]; f[:B]; f[B:]] of a batched [real; fake] D feature map (the
    real / mismatch / fake head inputs) in 2 copies; backward in one add and
    one copy instead of slice-backward zero fills, copies and adds."""

    @staticmethod
    def forward(ctx, feat, B):
        feat = to_nhwc_bf16(feat)
        N, C, H, W = feat.shape
        out = empty_nhwc(N + B, C, H, W, feat.device)
        out[:2 * B].unflatten(0, (2, B)).copy_(feat[:B].unsqueeze(0).expand(2, B, C, H, W))
        out[2 * B:].copy_(feat[B:])
        ctx.B, ctx.N = B, N
        return out

    @staticmethod
    def backward(ctx, g):
        B, N = ctx.B, ctx.N
        g = _as_bf16_grad(g)
        _, C, H, W = g.shape
        gf = empty_nhwc(N, C, H, W, g.device)
        torch.add(g[:B], g[B:2 * B], out=gf[:B])
        gf[B:].copy_(g[2 * B:])
        return gf, None


class BceLogitsFn(torch.autograd.Function):
    """F.binary_cross_entropy_with_logits(x, target) (mean)."""

    @staticmethod
    def forward(ctx, x, target):
        xc = x.float().contiguous()
        tc = target.float().contiguous()
        out = torch.empty((), dtype=F32, device=x.device)
        ops.bce_logits(xc.data_ptr(), tc.data_ptr(), xc.numel(), out.data_ptr(), stream())
        ctx.save_for_backward(xc, tc)
        ctx.shape = x.shape
        return out

    @staticmethod
    def backward(ctx, g):
        xc, tc = ctx.saved_tensors
        g = g.float().reshape(1).contiguous()
        dx = torch.empty_like(xc)
        ops.bce_logits_bwd(xc.data_ptr(), tc.data_ptr(), xc.numel(), g.data_ptr(), dx.data_ptr(), stream())
        return dx.reshape(ctx.shape), None


class GradPenaltyFn(torch.autograd.Function):
    """2 * mean_b ||[g_img_b, g_sent_b]||_2^6  (train.py:396-402)."""

    @staticmethod
    def forward(ctx, gx, gs):
        gx = to_nhwc_bf16(gx)
        gs = gs.float().reshape(gs.shape[0], -1).contiguous()
        N, C, H, W = gx.shape
        nrm2 = torch.empty(N, dtype=F32, device=gx.device)
        out = torch.empty((), dtype=F32, device=gx.device)
        ws = workspace(ops.gp_loss_workspace(N), gx.device)
        ops.gp_loss(gx.data_ptr(), ld_of(gx), N, H * W, C, gs.data_ptr(), gs.shape[1], nrm2.data_ptr(),
                    out.data_ptr(), ws.data_ptr(), stream())
        ctx.save_for_backward(gx, gs, nrm2)
        return out

    @staticmethod
    def backward(ctx, g):
        gx, gs, nrm2 = ctx.saved_tensors
        N, C, H, W = gx.shape
        g = g.float().reshape(1).contiguous()
        dgx = empty_nhwc(N, C, H, W, gx.device)
        dgs = torch.empty_like(gs)
        ops.gp_loss_bwd(gx.data_ptr(), ld_of(gx), N, H * W, C, gs.data_ptr(), gs.shape[1], nrm2.data_ptr(),
                        g.data_ptr(), dgx.data_ptr(), ld_of(dgx), dgs.data_ptr(), stream())
        return dgx, dgs


def _class_ids_dev(class_ids, device):
    if class_ids is None:
        return None
    t = torch.as_tensor(class_ids)
    return t.to(device=device, dtype=torch.long).contiguous()


class SimCEFn(torch.autograd.Function):
    """(CE(sim, labels), CE(sim^T, labels)) with same-class off-diagonal -inf masking
    (DAMSM_losses.py:238-245, 262-267, 326-338)."""

    @staticmethod
    def forward(ctx, sim, cls, labels=None):
        simc = sim.float().contiguous()
        B = simc.shape[0]
        out = torch.empty(2, dtype=F32, device=sim.device)
        ops.sim_ce(simc.data_ptr(), B, ptr(cls), ptr(labels), out.data_ptr(), stream())
        ctx.save_for_backward(simc, cls, labels)
        return out

    @staticmethod
    def backward(ctx, g):
        simc, cls, labels = ctx.saved_tensors
        g = g.float().contiguous()
        d = torch.empty_like(simc)
        ops.sim_ce_bwd(simc.data_ptr(), simc.shape[0], ptr(cls), ptr(labels), g.data_ptr(), d.data_ptr(), stream())
        return d, None, None


class WordsSimFn(torch.autograd.Function):
    """Word-level similarity block of words_loss (DAMSM_losses.py:281-331)
    before masking: sim[j][i] for this rank's images j (regions) x the given
    captions i (words, cap_lens -- all ranks' captions when data-parallel).
    `diag_off`: caption index of image 0's own caption (rank * B_local), used
    for the attention maps of the matching pairs."""

    MAX_WORDS = 32   # csrc/damsm.hip NW: one caption's words live in one workgroup's LDS / MFMA tiles

    @staticmethod
    def forward(ctx, regions, words, cap_lens, want_att, diag_off=0):
        # regions: (n_img, 256, 17, 17) fp32, NHWC-dense (the Inception projection output) or NCHW
        if words.shape[2] > WordsSimFn.MAX_WORDS:
            # the reference takes any words_num (DAMSM_losses.py:287-291); every shipped cfg has
            # TEXT.WORDS_NUM <= 20, and wider captions are refused rather than truncated
            raise ValueError('words_loss: captions of up to %d words are supported (got a %d-word batch; '
                             'cfg.TEXT.WORDS_NUM bounds it)' % (WordsSimFn.MAX_WORDS, words.shape[2]))
        n_img = regions.shape[0]
        if regions.dtype == F32 and T.is_nhwc(regions) and ld_of(regions) == regions.shape[1] \
                and regions.data_ptr() % 16 == 0:
            reg = regions
        else:
            reg = regions.float().permute(0, 2, 3, 1).contiguous().permute(0, 3, 1, 2)
        wd = words.float().contiguous()
        n_txt, Tn = wd.shape[0], wd.shape[2]
        lens = cap_lens.to(device=regions.device, dtype=torch.long).reshape(-1).contiguous()
        sim = torch.empty((n_img, n_txt), dtype=F32, device=regions.device)
        att = torch.zeros((n_img, Tn, 289) if want_att else (0,), dtype=F32, device=regions.device)
        # when a backward will follow, the workspace is sized for it and kept:
        # the backward reuses the operands prepared here
        bwd = bool(ctx.needs_input_grad[0] or ctx.needs_input_grad[1])
        ws = workspace(ops.words_workspace(n_img, n_txt, int(bwd), int(bool(ctx.needs_input_grad[1]))),
                       regions.device)
        ops.words_sim(reg.data_ptr(), wd.data_ptr(), lens.data_ptr(), n_img, n_txt, Tn, int(diag_off), sim.data_ptr(),
                      att.data_ptr() if want_att else 0, ws.data_ptr(), stream())
        ctx.ws = ws if bwd else None
        ctx.save_for_backward(reg, wd, lens)
        ctx.mark_non_differentiable(att)
        return sim, att

    @staticmethod
    def backward(ctx, dsim, _datt):
        reg, wd, lens = ctx.saved_tensors
        n_img, n_txt, Tn = reg.shape[0], wd.shape[0], wd.shape[2]
        dsim = dsim.float().contiguous()
        need_dw = ctx.needs_input_grad[1]
        dreg = torch.empty((n_img, 17, 17, 256), dtype=F32, device=dsim.device)
        dw = torch.empty_like(wd) if need_dw else None
        ws, prepared = ctx.ws, 1
        if ws is None or ws.numel() < ops.words_workspace(n_img, n_txt, 1, int(need_dw)):
            ws, prepared = workspace(ops.words_workspace(n_img, n_txt, 1, int(need_dw)), dsim.device), 0
        ops.words_sim_bwd(reg.data_ptr(), wd.data_ptr(), lens.data_ptr(), n_img, n_txt, Tn, dsim.data_ptr(),
                          dreg.data_ptr(), ptr(dw), ws.data_ptr(), prepared, stream())
        ctx.ws = None
        return dreg.permute(0, 3, 1, 2), dw, None, None, None


class GlobalAttentionFn(torch.autograd.Function):
    """GlobalAttentionGeneral.forward (DAMSM_losses.py:65-132) as one HIP
    launch (csrc/gag.hip): input (B, idf, ih, iw), context_key (B, idf, S),
    content_value (B, cdf, S), mask (B, S) bool or None ->
    (weightedContext (B, cdf, ih, iw), attn (B, S, ih, iw)); the mask is
    applied with the reference's ``mask.repeat(queryL, 1)`` row indexing."""

    @staticmethod
    def forward(ctx, inp, key, value, mask):
        B, idf, ih, iw = inp.shape
        Lq, S, cdf = ih * iw, key.shape[2], value.shape[1]
        x = inp.float().contiguous()
        k = key.float().contiguous()
        v = value.float().contiguous()
        m = mask.to(device=inp.device, dtype=torch.uint8).contiguous() if mask is not None else None
        wc = torch.empty((B, cdf, ih, iw), dtype=F32, device=inp.device)
        att = torch.empty((B, S, ih, iw), dtype=F32, device=inp.device)
        ws = workspace(ops.gag_fwd_workspace(B, Lq), inp.device)
        ops.gag_fwd(x.data_ptr(), k.data_ptr(), v.data_ptr(), ptr(m), B, idf, cdf, Lq, S, wc.data_ptr(),
                    att.data_ptr(), ws.data_ptr(), stream())
        ctx.save_for_backward(x, k, v, att)
        return wc, att

    @staticmethod
    def backward(ctx, dwc, datt):
        x, k, v, att = ctx.saved_tensors
        B, idf, ih, iw = x.shape
        Lq, S, cdf = ih * iw, k.shape[2], v.shape[1]
        dwc = dwc.float().contiguous() if dwc is not None else None
        datt = datt.float().contiguous() if datt is not None else None
        dx, dk, dv = torch.empty_like(x), torch.empty_like(k), torch.empty_like(v)
        ws = workspace(ops.gag_workspace(B, idf, cdf, Lq, S), x.device)
        ops.gag_bwd(x.data_ptr(), k.data_ptr(), v.data_ptr(), att.data_ptr(), ptr(dwc), ptr(datt), B, idf, cdf, Lq,
                    S, dx.data_ptr(), dk.data_ptr(), dv.data_ptr(), ws.data_ptr(), stream())
        return dx, dk, dv, None


class SentSimFn(torch.autograd.Function):
    """gamma3 * cos(cnn_a, rnn_b) for this rank's images a x the given
    captions b (DAMSM_losses.py:246-258)."""

    @staticmethod
    def forward(ctx, cnn, rnn):
        c = cnn.float().contiguous()
        r = rnn.float().contiguous()
        na, Dm = c.shape
        nb = r.shape[0]
        sim = torch.empty((na, nb), dtype=F32, device=c.device)
        ops.sent_sim(c.data_ptr(), r.data_ptr(), na, nb, Dm, sim.data_ptr(), stream())
        ctx.save_for_backward(c, r, sim)
        return sim

    @staticmethod
    def backward(ctx, dsim):
        c, r, sim = ctx.saved_tensors
        na, Dm = c.shape
        nb = r.shape[0]
        dsim = dsim.float().contiguous()
        nrm = torch.empty(na + nb, dtype=F32, device=c.device)
        dc = torch.empty_like(c) if ctx.needs_input_grad[0] else None
        dr = torch.empty_like(r) if ctx.needs_input_grad[1] else None
        ops.sent_sim_bwd(c.data_ptr(), r.data_ptr(), na, nb, Dm, sim.data_ptr(), dsim.data_ptr(), nrm.data_ptr(),
                         ptr(dc), ptr(dr), stream())
        return dc, dr


class AttrAttnFn(torch.autograd.Function):
    """softmax(q k^T) / sqrt(d) v over the 4 rows [sent; attrs] (models.py:161-169)."""

    @staticmethod
    def forward(ctx, q, k, v, scale):
        q, k, v = q.float().contiguous(), k.float().contiguous(), v.float().contiguous()
        B, L, Dm = q.shape
        probs = torch.empty((B, L, L), dtype=F32, device=q.device)
        out = torch.empty_like(q)
        ops.attr_attn(q.data_ptr(), k.data_ptr(), v.data_ptr(), B, L, Dm, scale, probs.data_ptr(), out.data_ptr(), 0,
                      stream())
        ctx.scale = scale
        ctx.save_for_backward(q, k, v, probs)
        return out

    @staticmethod
    def backward(ctx, g):
        q, k, v, probs = ctx.saved_tensors
        B, L, Dm = q.shape
        g = g.float().contiguous()
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        ops.attr_attn_bwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), probs.data_ptr(), g.data_ptr(), B, L, Dm,
                          ctx.scale, dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), stream())
        return dq, dk, dv, None


def class_onehot(class_ids, B, ncls, device):
    ids = _class_ids_dev(class_ids, device)
    out = torch.empty((B, ncls), dtype=F32, device=device)
    err = torch.zeros(1, dtype=torch.int32, device=device)
    ops.class_onehot(ids.data_ptr(), B, ncls, out.data_ptr(), err.data_ptr(), stream())
    return out, err


def _commit_after_backward(cls):
    f = cls.backward

    def backward(ctx, *grads):
        out = f(ctx, *grads)
        if _PENDING_SINKS:
            _commit_sinks()
        return out
    backward.__doc__ = f.__doc__
    cls.backward = staticmethod(backward)


# every Function of this module: a bucket completed by the direct gradient
# writes of a backward is reduced once that backward has launched them all
for _cls in list(globals().values()):
    if isinstance(_cls, type) and issubclass(_cls, torch.autograd.Function) and _cls.__module__ == __name__ \
            and 'backward' in _cls.__dict__:
        _commit_after_backward(_cls)
