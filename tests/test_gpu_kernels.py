"""Kernel-level parity: every HIP op (through the C ABI) against a plain
PyTorch fp32 CPU reference of the same op on the same bf16-rounded inputs.

Tolerances: bf16 storage of activations/gradients with fp32 accumulation ->
relative L2 error <= 1e-2 (outputs rounded once to bf16: ~2e-3 expected);
integer / label work bit-exact."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from _util import rel_l2, conv_knob  # noqa: E402


def _bf(t):
    return t.to(torch.bfloat16).float()


def _mods():
    from eegan_hip import functional as Fn
    from eegan_hip import tensor as T
    from eegan_hip.nn import Conv2d
    return Fn, T, Conv2d


def _nhwc(x, dev):
    """fp32 NCHW CPU -> bf16 NHWC device activation (padded ld for C >= 8)."""
    Fn, T, _ = _mods()
    N, C, H, W = x.shape
    t = T.empty_nhwc(N, C, H, W, dev)
    t.copy_(x.to(dev).to(torch.bfloat16))
    return t


CONV_CASES = [
    # N, Cin, H, W, Cout, k, stride, pad, bias, act, up2
    (2, 32, 16, 16, 64, 3, 1, 1, False, None, False),
    (2, 64, 16, 16, 32, 4, 2, 1, False, 'lrelu', False),
    (2, 3, 32, 32, 16, 3, 1, 1, True, None, False),
    (2, 16, 8, 8, 3, 3, 1, 1, False, 'tanh', False),
    (2, 100, 8, 8, 1, 1, 1, 0, False, None, False),
    (2, 24, 8, 8, 100, 3, 1, 1, False, 'relu', False),
    (2, 64, 8, 8, 64, 4, 4, 0, True, None, False),
    (3, 32, 4, 4, 1, 4, 1, 0, False, None, False),
    (2, 32, 8, 8, 16, (1, 7), 1, (0, 3), False, 'relu', False),
    (2, 32, 17, 17, 48, 3, 2, 0, False, None, False),
    (2, 32, 8, 8, 32, 3, 1, 1, False, None, True),
    (2, 16, 8, 8, 24, 1, 1, 0, True, None, True),
    (4, 128, 32, 32, 256, 3, 1, 1, False, 'lrelu', False),
    (2, 48, 9, 9, 40, 3, 1, 1, False, None, False),
    # many pixel splits of the weight gradient; odd widths (pixel walk wraps rows mid-step)
    (8, 32, 64, 64, 32, 3, 1, 1, True, None, False),
    (2, 32, 37, 23, 64, 4, 2, 1, False, 'lrelu', False),
    # small grids: split-K forward / backward-data with the hoisted-gather kernel
    (2, 256, 4, 4, 192, 3, 1, 1, True, 'lrelu', False),
    (2, 96, 6, 10, 64, 4, 2, 1, False, None, False),
]


def test_conv_fast_path_matches_generic(gpu, monkeypatch):
    """The hoisted-gather kernels (EEGAN_CONV fast=1, default: forward,
    backward-data, weight gradient) sum the same products in the same order as
    the generic pipelined kernels: bit-identical."""
    Fn, T, _ = _mods()
    for N, Cin, H, W, Cout, k, st, pad in [(2, 64, 12, 20, 96, 3, 1, 1), (2, 48, 16, 16, 32, 4, 2, 1),
                                            (2, 256, 4, 4, 128, 3, 1, 1), (3, 40, 8, 8, 72, 3, 1, 1),
                                            (3, 24, 4, 4, 48, 4, 4, 0), (2, 32, 64, 64, 64, 4, 2, 1)]:
        torch.manual_seed(N * Cin + H)
        g = Fn.Geom(Cout, k, k, st, pad, pad, 0)
        x = _nhwc(torch.randn(N, Cin, H, W), gpu)
        Wt = (torch.randn(Cout, Cin, k, k) * 0.05).to(gpu)
        Ho, Wo = g.out_hw(H, W)
        dz = _nhwc(torch.randn(N, Cout, Ho, Wo), gpu)
        outs = []
        for fast in ('0', '1'):
            conv_knob(monkeypatch, 'fast', fast)
            outs.append((Fn.conv_fwd_raw(x, Wt, None, g).float().cpu(),
                         Fn.conv_bwd_data_raw(dz, Wt, g, tuple(x.shape)).float().cpu(),
                         Fn.conv_bwd_weight_raw(x, dz, g, Wt.shape).cpu()))
        for a, b in zip(*outs):
            assert torch.equal(a, b)


def test_conv_thin_path_matches_tile(gpu, monkeypatch):
    """3x3 stride-1 convs with <= 32 output rows (stem, get_image, 32-channel
    256x256 convs and their data gradients) take the weight-stationary thin
    kernel (EEGAN_CONV thin=1, default): same K steps in the same order as the
    tile kernels, so bit-identical; also checked against torch fp32."""
    Fn, T, _ = _mods()
    for N, Cin, H, W, Cout, pad, up2, bias, act in [
            (2, 3, 20, 24, 32, 1, 0, True, 0), (2, 32, 20, 24, 3, 1, 0, False, 3),
            (2, 32, 17, 15, 32, 1, 0, False, 2), (3, 64, 9, 13, 16, 1, 0, False, 0),
            (2, 32, 13, 11, 32, 0, 0, False, 0), (2, 32, 16, 20, 24, 1, 1, False, 1),
            (1, 5, 7, 9, 12, 1, 0, True, 0),
            # OW % 64 == 0: the LDS halo-tile variant (partial last tile row: H % 8 != 0)
            (2, 3, 13, 128, 32, 1, 0, True, 0), (2, 32, 10, 64, 3, 1, 0, False, 3),
            (1, 32, 16, 64, 32, 1, 0, False, 2), (1, 32, 11, 66, 20, 0, 0, False, 0),
            (1, 32, 16, 128, 32, 1, 1, False, 1), (1, 7, 8, 64, 16, 1, 0, False, 0)]:
        torch.manual_seed(N * Cin + H + Cout)
        g = Fn.Geom(Cout, 3, 3, 1, pad, pad, up2)
        xl = torch.randn(N, Cin, H // 2 if up2 else H, W // 2 if up2 else W)
        x = _nhwc(xl, gpu)
        Wt = _bf(torch.randn(Cout, Cin, 3, 3) * 0.1).to(gpu)
        b = torch.randn(Cout).to(gpu) if bias else None
        Ho, Wo = g.out_hw(H, W)
        dz = _nhwc(torch.randn(N, Cout, Ho, Wo), gpu)
        outs = []
        for thin in ('0', '1'):
            conv_knob(monkeypatch, 'thin', thin)
            o = [Fn.conv_fwd_raw(x, Wt, b, g, act=act).float().cpu()]
            if not up2:
                o.append(Fn.conv_bwd_data_raw(dz, Wt, g, tuple(x.shape)).float().cpu())
            outs.append(o)
        for a, c in zip(*outs):
            assert torch.equal(a, c)
        xin = F.interpolate(_bf(xl), scale_factor=2) if up2 else _bf(xl)
        yr = F.conv2d(xin, Wt.cpu(), None if b is None else b.cpu(), 1, pad)
        yr = {0: yr, 1: F.relu(yr), 2: F.leaky_relu(yr, 0.2), 3: torch.tanh(yr)}[act]
        assert rel_l2(outs[1][0], yr) < 1e-2
        if not up2:
            xr = xin.clone().requires_grad_()
            F.conv2d(xr, Wt.cpu(), None, 1, pad).backward(dz.float().cpu())
            assert rel_l2(outs[1][1], xr.grad) < 1e-2


def test_conv_thin_wgrad(gpu, monkeypatch):
    """Weight gradient of 3x3 convs with <= 8 output and 25..64 input channels
    (get_image) through the transposed-read thin kernel: against torch fp32
    and the tile path (different fp32 summation order, so within 1e-5)."""
    Fn, T, _ = _mods()
    for N, Cin, H, W, Cout in [(2, 32, 8, 64, 3), (1, 32, 12, 128, 8), (2, 28, 4, 64, 5), (4, 32, 8, 64, 1),
                               (2, 64, 8, 64, 3), (1, 56, 4, 128, 6)]:
        torch.manual_seed(N + Cin + H + Cout)
        g = Fn.Geom(Cout, 3, 3, 1, 1, 1, 0)
        xl = _bf(torch.randn(N, Cin, H, W))
        dzl = _bf(torch.randn(N, Cout, H, W))
        x, dz = _nhwc(xl, gpu), _nhwc(dzl, gpu)
        outs = []
        for thin in ('0', '1'):
            conv_knob(monkeypatch, 'thin', thin)
            outs.append(Fn.conv_bwd_weight_raw(x, dz, g, (Cout, Cin, 3, 3)).cpu())
        wr = torch.zeros(Cout, Cin, 3, 3, requires_grad=True)
        F.conv2d(xl, wr, None, 1, 1).backward(dzl)
        assert rel_l2(outs[1], wr.grad) < 1e-4
        assert torch.allclose(outs[0], outs[1], rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize('blocks', ['0', '16'])
def test_conv_wgrad_halo3(gpu, monkeypatch, blocks):
    """Weight gradient of 3x3 / stride-1 convs with 32 / 64 input channels and
    32-channel output tiles on the halo-staged kernel (conv_wgrad_halo3_kernel,
    EEGAN_CONV wgrad_halo=1, default) against torch fp32 and the tile path
    (wgrad_halo=0; another fp32 summation order): one, two and three output
    tiles, blocks with several tiles (wgrad_halo_blocks=16) and blocks past the
    last tile (their zero partials), accumulation into an existing gradient."""
    Fn, T, _ = _mods()
    if blocks != '0':
        conv_knob(monkeypatch, 'wgrad_halo_blocks', blocks)
    for N, Cin, H, W, Cout in [(2, 32, 8, 64, 32), (1, 64, 12, 128, 64), (2, 32, 4, 32, 64), (3, 64, 8, 32, 32),
                               (2, 64, 16, 64, 96)]:
        torch.manual_seed(N + Cin + H + Cout)
        g = Fn.Geom(Cout, 3, 3, 1, 1, 1, 0)
        xl = _bf(torch.randn(N, Cin, H, W))
        dzl = _bf(torch.randn(N, Cout, H, W))
        x, dz = _nhwc(xl, gpu), _nhwc(dzl, gpu)
        outs = []
        for on in ('0', '1'):
            conv_knob(monkeypatch, 'wgrad_halo', on)
            outs.append(Fn.conv_bwd_weight_raw(x, dz, g, (Cout, Cin, 3, 3)).cpu())
        wr = torch.zeros(Cout, Cin, 3, 3, requires_grad=True)
        F.conv2d(xl, wr, None, 1, 1).backward(dzl)
        assert rel_l2(outs[1], wr.grad) < 1e-4, (N, Cin, H, Cout)
        assert torch.allclose(outs[0], outs[1], rtol=1e-5, atol=1e-4)
        conv_knob(monkeypatch, 'wgrad_halo', '1')
        base = (torch.randn(Cout, Cin, 3, 3) * 0.1).to(gpu).contiguous(memory_format=torch.channels_last)
        acc = base.clone()
        Fn.conv_bwd_weight_raw(x, dz, g, (Cout, Cin, 3, 3), out=acc)
        assert torch.allclose(acc.cpu(), base.cpu() + outs[1], rtol=1e-5, atol=1e-4)


def test_conv_thin_wgrad_channel_groups(gpu, monkeypatch):
    """The thin weight-gradient kernel for up to 64 output channels, in
    8-channel groups on the grid's y axis (EEGAN_CONV wgrad_thin_maxk): against
    torch fp32 and the tile path; a ragged last group (Cout % 8 != 0) and a
    padded dy row (its channels past Cout are never read into written rows)."""
    Fn, T, _ = _mods()
    conv_knob(monkeypatch, 'wgrad_thin_maxk', '64')
    for N, Cin, H, W, Cout in [(2, 32, 8, 64, 32), (1, 64, 12, 128, 64), (2, 32, 4, 64, 36), (2, 28, 8, 64, 16),
                               (1, 64, 8, 64, 20)]:
        torch.manual_seed(N + Cin + H + Cout)
        g = Fn.Geom(Cout, 3, 3, 1, 1, 1, 0)
        xl = _bf(torch.randn(N, Cin, H, W))
        dzl = _bf(torch.randn(N, Cout, H, W))
        x, dz = _nhwc(xl, gpu), _nhwc(dzl, gpu)
        outs = []
        for thin in ('0', '1'):
            conv_knob(monkeypatch, 'thin', thin)
            outs.append(Fn.conv_bwd_weight_raw(x, dz, g, (Cout, Cin, 3, 3)).cpu())
        wr = torch.zeros(Cout, Cin, 3, 3, requires_grad=True)
        F.conv2d(xl, wr, None, 1, 1).backward(dzl)
        assert rel_l2(outs[1], wr.grad) < 1e-4, (N, Cin, H, Cout)
        assert torch.allclose(outs[0], outs[1], rtol=1e-5, atol=1e-4)


def test_splitk_reduce_vector_path_bit_identical(gpu, monkeypatch):
    """The split-K reduce's 4-channel vector path (default) against the scalar
    path (EEGAN_CONV red_vec4=0): same summation order, so torch.equal, over
    forward (bias, act, residual + gain) and backward-data (activation gate,
    half-resolution residual of resD's pooled shortcut) epilogues; odd channel
    counts take the scalar path in both runs.  EEGAN_CONV target= forces the
    K split on these small grids."""
    Fn, T, _ = _mods()
    monkeypatch.setattr(Fn, 'SPLITK_FUSED', True)   # counters off by default (the reduce launch is)
    conv_knob(monkeypatch, 'target', '4096')
    conv_knob(monkeypatch, 'mink', '2')
    lrelu = Fn.ACT_CODES['lrelu']
    for N, Cin, H, W, Cout, k, st, pad in [(2, 256, 4, 4, 128, 3, 1, 1), (2, 96, 8, 8, 64, 4, 2, 1),
                                            (3, 128, 6, 6, 36, 3, 1, 1), (2, 64, 8, 8, 9, 4, 2, 1),
                                            (2, 9, 8, 8, 64, 3, 1, 1)]:
        torch.manual_seed(N * Cin + Cout)
        g = Fn.Geom(Cout, k, k, st, pad, pad, 0)
        x = _nhwc(torch.randn(N, Cin, H, W), gpu)
        Wt = (torch.randn(Cout, Cin, k, k) * 0.05).to(gpu)
        b = torch.randn(Cout).to(gpu)
        gam = torch.tensor([0.7]).to(gpu)
        Ho, Wo = g.out_hw(H, W)
        res = _nhwc(torch.randn(N, Cout, Ho, Wo), gpu)
        dz = _nhwc(torch.randn(N, Cout, Ho, Wo), gpu)
        gate = _nhwc(torch.randn(N, Cin, H, W), gpu)
        halfres = _nhwc(torch.randn(N, Cin, H // 2, W // 2), gpu)
        outs = []
        for vec in ('0', '1'):
            conv_knob(monkeypatch, 'red_vec4', vec)
            o = [Fn.conv_fwd_raw(x, Wt, b, g, act=lrelu, res=res, gamma=gam).float().cpu(),
                 Fn.conv_fwd_raw(x, Wt, b, g, act=lrelu, out_f32=True).cpu(),
                 Fn.conv_bwd_data_raw(dz, Wt, g, tuple(x.shape), gate=gate, gate_act=lrelu).float().cpu(),
                 Fn.conv_bwd_data_raw(dz, Wt, g, tuple(x.shape), res=halfres, res_up2=1, res_scale=0.25).float().cpu()]
            outs.append(o)
        for a, c in zip(*outs):
            assert torch.equal(a, c)


def test_splitk_fused_finish_bit_identical(gpu, monkeypatch):
    """The in-kernel split-K finish (eegan_conv_desc.splitk_ctr; the last-
    arriving split of each tile sums the sc1-written partials in split order)
    against the separate reduce launch (EEGAN_CONV splitk_fused=0): torch.equal
    over forward and backward-data epilogues (bias / act / residual, gate,
    half-resolution residual, stride-2 parity classes), repeated launches and
    two streams at once; every counter is back at zero afterwards."""
    Fn, T, _ = _mods()
    monkeypatch.setattr(Fn, 'SPLITK_FUSED', True)   # counters off by default (the reduce launch is)
    conv_knob(monkeypatch, 'target', '4096')
    conv_knob(monkeypatch, 'mink', '2')
    lrelu = Fn.ACT_CODES['lrelu']

    def run(x, Wt, b, g, gam, res, dz, gate, halfres):
        return [Fn.conv_fwd_raw(x, Wt, b, g, act=lrelu, res=res, gamma=gam).float().cpu(),
                Fn.conv_fwd_raw(x, Wt, b, g, act=lrelu, out_f32=True).cpu(),
                Fn.conv_bwd_data_raw(dz, Wt, g, tuple(x.shape), gate=gate, gate_act=lrelu).float().cpu(),
                Fn.conv_bwd_data_raw(dz, Wt, g, tuple(x.shape), res=halfres, res_up2=1, res_scale=0.25).float().cpu()]

    side = torch.cuda.Stream()
    for N, Cin, H, W, Cout, k, st, pad in [(2, 256, 4, 4, 128, 3, 1, 1), (2, 96, 8, 8, 64, 4, 2, 1),
                                            (16, 512, 4, 4, 512, 3, 1, 1), (4, 512, 8, 8, 512, 4, 2, 1)]:
        torch.manual_seed(N * Cin + Cout)
        g = Fn.Geom(Cout, k, k, st, pad, pad, 0)
        x = _nhwc(torch.randn(N, Cin, H, W), gpu)
        Wt = (torch.randn(Cout, Cin, k, k) * 0.05).to(gpu)
        b = torch.randn(Cout).to(gpu)
        gam = torch.tensor([0.7]).to(gpu)
        Ho, Wo = g.out_hw(H, W)
        args = (x, Wt, b, g, gam, _nhwc(torch.randn(N, Cout, Ho, Wo), gpu), _nhwc(torch.randn(N, Cout, Ho, Wo), gpu),
                _nhwc(torch.randn(N, Cin, H, W), gpu), _nhwc(torch.randn(N, Cin, H // 2, W // 2), gpu))
        conv_knob(monkeypatch, 'splitk_fused', '0')
        ref = run(*args)
        conv_knob(monkeypatch, 'splitk_fused', '1')
        for rep in range(2):
            for a_, c_ in zip(ref, run(*args)):
                assert torch.equal(a_, c_), (N, Cin, Cout, k, rep)
        with torch.cuda.stream(side):   # a second lane with its own counters, concurrently
            side.wait_stream(torch.cuda.default_stream())
            o_side = run(*args)
        o_main = run(*args)
        torch.cuda.synchronize()
        for a_, c_, e_ in zip(ref, o_side, o_main):
            assert torch.equal(a_, c_) and torch.equal(a_, e_)
    assert len(Fn._SPLITK_CTR) >= 2
    for ctr in Fn._SPLITK_CTR.values():
        assert int(ctr.abs().sum()) == 0


@pytest.mark.parametrize('target', ['512', '4096'])
def test_conv_wide_stages_bit_identical(gpu, monkeypatch, target):
    """Wide pair stages (one 64-channel stage of whole 128-B lines per K-step
    pair, EEGAN_CONV wide=1, default) against two 32-channel stages (=0): same
    K order and MFMA sequence, so torch.equal -- forward with bias / act /
    residual + gain and fp32 out, backward-data with gate, the
    half-resolution residual and stride-2 parity classes, channel counts with
    padded 64-channel pairs (72, 200), with and without split-K."""
    Fn, T, _ = _mods()
    conv_knob(monkeypatch, 'target', target)
    conv_knob(monkeypatch, 'mink', '2')
    lrelu = Fn.ACT_CODES['lrelu']
    for N, Cin, H, W, Cout, k, st, pad in [(2, 64, 16, 16, 128, 3, 1, 1), (3, 128, 9, 11, 64, 3, 1, 1),
                                            (2, 96, 16, 16, 256, 4, 2, 1), (2, 64, 12, 12, 200, 1, 1, 0),
                                            (4, 256, 8, 8, 72, 3, 1, 1), (2, 128, 16, 16, 96, 4, 2, 1),
                                            (2, 72, 10, 10, 128, 3, 1, 1), (2, 200, 8, 8, 64, 3, 1, 1),
                                            (2, 32, 32, 32, 64, 4, 2, 1), (2, 24, 16, 16, 64, 3, 1, 1)]:
        torch.manual_seed(N * Cin + Cout + H)
        g = Fn.Geom(Cout, k, k, st, pad, pad, 0)
        x = _nhwc(torch.randn(N, Cin, H, W), gpu)
        Wt = (torch.randn(Cout, Cin, k, k) * 0.05).to(gpu)
        b = torch.randn(Cout).to(gpu)
        gam = torch.tensor([0.7]).to(gpu)
        Ho, Wo = g.out_hw(H, W)
        res = _nhwc(torch.randn(N, Cout, Ho, Wo), gpu)
        dz = _nhwc(torch.randn(N, Cout, Ho, Wo), gpu)
        gate = _nhwc(torch.randn(N, Cin, H, W), gpu)
        halfres = _nhwc(torch.randn(N, Cin, H // 2, W // 2), gpu) if H % 2 == 0 and W % 2 == 0 else None
        outs = []
        for wide in ('0', '1'):
            conv_knob(monkeypatch, 'wide', wide)
            o = [Fn.conv_fwd_raw(x, Wt, b, g, act=lrelu, res=res, gamma=gam).float().cpu(),
                 Fn.conv_fwd_raw(x, Wt, b, g, act=lrelu, out_f32=True).cpu(),
                 Fn.conv_bwd_data_raw(dz, Wt, g, tuple(x.shape), gate=gate, gate_act=lrelu).float().cpu()]
            if halfres is not None:
                o.append(Fn.conv_bwd_data_raw(dz, Wt, g, tuple(x.shape), res=halfres, res_up2=1,
                                              res_scale=0.25).float().cpu())
            outs.append(o)
        for a, c in zip(*outs):
            assert torch.equal(a, c), (N, Cin, H, W, Cout, k, st)


def test_conv_s2bwd_halo_bit_identical(gpu, monkeypatch):
    """4x4 / stride-2 / pad-1 data gradients with <= 64 input channels (resD
    block0's and block1's conv_r[0]) take the shared-halo parity-class kernel
    (EEGAN_CONV s2b=1, default): same K order as the unsplit tile kernel
    (EEGAN_CONV target=1 keeps it unsplit), so torch.equal -- plain, gated and
    with the half-resolution pooled-shortcut residual; 16..64 input (one or two
    32-row slices) and 32/64/128 output channels, one- and multi-tile grids;
    also against torch fp32."""
    Fn, T, _ = _mods()
    conv_knob(monkeypatch, 'target', '1')
    lrelu = Fn.ACT_CODES['lrelu']
    for N, Cin, H, W, Cout in [(2, 32, 64, 64, 64), (3, 16, 8, 64, 32), (1, 24, 16, 128, 64),
                               (2, 32, 24, 192, 32), (5, 32, 8, 64, 64),
                               # two 32-row slices of the input channels, 128-channel K runs (block1)
                               (2, 64, 16, 64, 128), (1, 48, 8, 128, 128), (2, 64, 8, 64, 64), (1, 40, 8, 64, 32)]:
        torch.manual_seed(N * Cin + Cout + H)
        g = Fn.Geom(Cout, 4, 4, 2, 1, 1, 0)
        Wt = _bf(torch.randn(Cout, Cin, 4, 4) * 0.05)
        Ho, Wo = g.out_hw(H, W)
        dzl = _bf(torch.randn(N, Cout, Ho, Wo))
        dz = _nhwc(dzl, gpu)
        gate = _nhwc(torch.randn(N, Cin, H, W), gpu)
        halfres = _nhwc(torch.randn(N, Cin, H // 2, W // 2), gpu)
        outs = []
        for s2b in ('0', '1'):
            conv_knob(monkeypatch, 's2b', s2b)
            outs.append([Fn.conv_bwd_data_raw(dz, Wt.to(gpu), g, (N, Cin, H, W)).float().cpu(),
                         Fn.conv_bwd_data_raw(dz, Wt.to(gpu), g, (N, Cin, H, W), gate=gate,
                                              gate_act=lrelu).float().cpu(),
                         Fn.conv_bwd_data_raw(dz, Wt.to(gpu), g, (N, Cin, H, W), res=halfres, res_up2=1,
                                              res_scale=0.25).float().cpu()])
        for a, c in zip(*outs):
            assert torch.equal(a, c), (N, Cin, H, W, Cout)
        xr = torch.zeros(N, Cin, H, W, requires_grad=True)
        F.conv2d(xr, Wt, None, 2, 1).backward(dzl)
        assert rel_l2(outs[1][0], xr.grad) < 1e-2


def test_conv_1x1_stream_bit_identical(gpu, monkeypatch):
    """1x1 convs with <= 256 packed K columns (resD's conv_s, get_mask's
    100 -> 1 projection) and their data gradients take the streaming pointwise
    kernel (EEGAN_CONV 1x1=1, default): same K order as the unsplit tile kernel
    (EEGAN_CONV target=1), so torch.equal -- forward with bias / act / residual
    + gain and fp32 out, backward-data plain, gated and with the
    half-resolution residual; channel counts that straddle a 16-B chunk (100),
    one-channel operands (the packed 8-channel K row) and several output-row
    slices per pixel group; also against torch fp32."""
    Fn, T, _ = _mods()
    conv_knob(monkeypatch, 'target', '1')
    lrelu = Fn.ACT_CODES['lrelu']
    for N, Cin, H, W, Cout in [(2, 32, 16, 24, 64), (3, 64, 8, 8, 128), (2, 100, 12, 10, 1), (2, 1, 8, 8, 100),
                               (2, 256, 4, 4, 512), (1, 128, 6, 6, 256), (2, 24, 5, 7, 40), (2, 200, 4, 4, 72)]:
        torch.manual_seed(N * Cin + Cout + H)
        g = Fn.Geom(Cout, 1, 1, 1, 0, 0, 0)
        xl = _bf(torch.randn(N, Cin, H, W))
        x = _nhwc(xl, gpu)
        Wt = _bf(torch.randn(Cout, Cin, 1, 1) * 0.1)
        b = torch.randn(Cout).to(gpu)
        gam = torch.tensor([0.7]).to(gpu)
        res = _nhwc(torch.randn(N, Cout, H, W), gpu)
        dzl = _bf(torch.randn(N, Cout, H, W))
        dz = _nhwc(dzl, gpu)
        gate = _nhwc(torch.randn(N, Cin, H, W), gpu)
        even = H % 2 == 0 and W % 2 == 0
        halfres = _nhwc(torch.randn(N, Cin, H // 2, W // 2), gpu) if even else None
        Wd = Wt.to(gpu)
        outs = []
        for on in ('0', '1'):
            conv_knob(monkeypatch, '1x1', on)
            o = [Fn.conv_fwd_raw(x, Wd, b, g, act=lrelu, res=res, gamma=gam).float().cpu(),
                 Fn.conv_fwd_raw(x, Wd, b, g, act=lrelu, out_f32=True).cpu(),
                 Fn.conv_fwd_raw(x, Wd, None, g).float().cpu(),
                 Fn.conv_bwd_data_raw(dz, Wd, g, (N, Cin, H, W)).float().cpu(),
                 Fn.conv_bwd_data_raw(dz, Wd, g, (N, Cin, H, W), gate=gate, gate_act=lrelu).float().cpu()]
            if halfres is not None:
                o.append(Fn.conv_bwd_data_raw(dz, Wd, g, (N, Cin, H, W), res=halfres, res_up2=1,
                                              res_scale=0.25).float().cpu())
            outs.append(o)
        for a, c in zip(*outs):
            assert torch.equal(a, c), (N, Cin, H, W, Cout)
        assert rel_l2(outs[1][2], F.conv2d(xl, Wt)) < 1e-2
        xr = xl.clone().requires_grad_()
        F.conv2d(xr, Wt).backward(dzl)
        assert rel_l2(outs[1][3], xr.grad) < 1e-2


@pytest.mark.parametrize('target', ['1', '512'])
def test_conv_staged_epilogue_bit_identical(gpu, monkeypatch, target):
    """The tile kernel's LDS-staged epilogue (EEGAN_CONV stage_epi=1, default:
    whole 16-B runs of 8 channels per thread) against the direct MFMA-layout
    epilogue (=0): same arithmetic in the same order, so torch.equal --
    forward with bias / act / residual + gain, backward-data with the gate,
    the half-resolution residual and stride-2 parity classes, every tile
    shape (16..128 rows x 64..256 pixels), ragged pixel tails; split-K and
    unaligned cases keep the direct epilogue in both runs."""
    Fn, T, _ = _mods()
    conv_knob(monkeypatch, 'target', target)
    lrelu = Fn.ACT_CODES['lrelu']
    for N, Cin, H, W, Cout, k, st, pad in [(2, 64, 16, 16, 128, 3, 1, 1), (3, 128, 9, 11, 64, 3, 1, 1),
                                            (2, 96, 16, 16, 256, 4, 2, 1), (2, 64, 12, 12, 200, 1, 1, 0),
                                            (4, 256, 8, 8, 72, 3, 1, 1), (2, 128, 16, 16, 96, 4, 2, 1),
                                            (2, 48, 32, 32, 32, 3, 1, 1), (2, 32, 33, 31, 16, 3, 1, 1),
                                            (2, 64, 32, 32, 64, 4, 2, 1), (2, 24, 16, 16, 40, 3, 1, 1),
                                            (1, 512, 4, 4, 512, 3, 1, 1), (2, 40, 16, 16, 24, 4, 2, 1)]:
        torch.manual_seed(N * Cin + Cout + H)
        g = Fn.Geom(Cout, k, k, st, pad, pad, 0)
        x = _nhwc(torch.randn(N, Cin, H, W), gpu)
        Wt = (torch.randn(Cout, Cin, k, k) * 0.05).to(gpu)
        b = torch.randn(Cout).to(gpu)
        gam = torch.tensor([0.7]).to(gpu)
        Ho, Wo = g.out_hw(H, W)
        res = _nhwc(torch.randn(N, Cout, Ho, Wo), gpu)
        dz = _nhwc(torch.randn(N, Cout, Ho, Wo), gpu)
        gate = _nhwc(torch.randn(N, Cin, H, W), gpu)
        halfres = _nhwc(torch.randn(N, Cin, H // 2, W // 2), gpu) if H % 2 == 0 and W % 2 == 0 else None
        outs = []
        for on in ('0', '1'):
            conv_knob(monkeypatch, 'stage_epi', on)
            o = [Fn.conv_fwd_raw(x, Wt, b, g, act=lrelu, res=res, gamma=gam).float().cpu(),
                 Fn.conv_fwd_raw(x, Wt, None, g).float().cpu(),
                 Fn.conv_bwd_data_raw(dz, Wt, g, tuple(x.shape)).float().cpu(),
                 Fn.conv_bwd_data_raw(dz, Wt, g, tuple(x.shape), gate=gate, gate_act=lrelu).float().cpu()]
            if halfres is not None:
                o.append(Fn.conv_bwd_data_raw(dz, Wt, g, tuple(x.shape), res=halfres, res_up2=1,
                                              res_scale=0.25).float().cpu())
            outs.append(o)
        for a, c in zip(*outs):
            assert torch.equal(a, c), (N, Cin, H, W, Cout, k, st)


def _nhwc_nan_padded(x, dev):
    """As _nhwc, with every padding channel of the row (ld > C) holding NaN bits."""
    Fn, T, _ = _mods()
    N, C, H, W = x.shape
    t = T.empty_nhwc(N, C, H, W, dev)
    torch.empty(0, dtype=torch.uint8, device=dev).set_(t.untyped_storage()).fill_(255)
    t.copy_(x.to(dev).to(torch.bfloat16))
    return t


def test_conv_ragged_channels_lds_path(gpu, monkeypatch):
    """Operands whose channel count is not a multiple of 8 (get_mask's 100
    channels, models.py:35-41) take the LDS-DMA kernels (hoisted-gather fast
    kernel, or conv_glds_kernel with EEGAN_CONV fast=0) with the straddling
    16-B chunk masked per K-step (EEGAN_CONV glds_ragged=1, default) instead of
    the register-staged kernel (=0): same K order, so torch.equal -- even with
    NaN bits in the padding channels -- and against torch fp32."""
    Fn, T, _ = _mods()
    conv_knob(monkeypatch, 'target', '1')
    for N, Cin, H, W, Cout, k, st, pad in [(2, 64, 16, 16, 100, 3, 1, 1), (2, 100, 12, 12, 64, 3, 1, 1),
                                            (2, 20, 16, 16, 36, 4, 2, 1), (1, 128, 8, 8, 100, 3, 1, 1),
                                            (2, 44, 9, 11, 52, 3, 1, 1)]:
        torch.manual_seed(N * Cin + Cout + H)
        g = Fn.Geom(Cout, k, k, st, pad, pad, 0)
        xl = _bf(torch.randn(N, Cin, H, W))
        x = _nhwc_nan_padded(xl, gpu)
        Wt = _bf(torch.randn(Cout, Cin, k, k) * 0.05)
        Wd = Wt.to(gpu)
        Ho, Wo = g.out_hw(H, W)
        dzl = _bf(torch.randn(N, Cout, Ho, Wo))
        dz = _nhwc_nan_padded(dzl, gpu)
        outs = []
        for rag, fast in (('0', '1'), ('1', '0'), ('1', '1')):
            conv_knob(monkeypatch, 'glds_ragged', rag)
            conv_knob(monkeypatch, 'fast', fast)
            outs.append([Fn.conv_fwd_raw(x, Wd, None, g).float().cpu(),
                         Fn.conv_bwd_data_raw(dz, Wd, g, (N, Cin, H, W)).float().cpu()])
        for other in outs[1:]:
            for a, c in zip(outs[0], other):
                assert torch.isfinite(c).all()
                assert torch.equal(a, c), (N, Cin, H, W, Cout, k, st)
        assert rel_l2(outs[1][0], F.conv2d(xl, Wt, None, st, pad)) < 1e-2
        xr = xl.clone().requires_grad_()
        F.conv2d(xr, Wt, None, st, pad).backward(dzl)
        assert rel_l2(outs[1][1], xr.grad) < 1e-2


def test_cat_channels(gpu):
    """Inception branch concat (one launch when every part has C % 8 == 0,
    else the per-part path) against torch.cat, with strided (sliced) parts."""
    Fn, T, _ = _mods()
    torch.manual_seed(5)
    for Cs in [(64, 64, 96, 32), (320, 384, 384, 384, 384, 192), (8, 12, 16)]:
        src = [torch.randn(3, c, 5, 7) for c in Cs]
        parts = []
        for i, t in enumerate(src):
            if i == 1:  # a channel slice of a wider NHWC buffer (ld > C)
                big = _nhwc(torch.randn(3, t.shape[1] + 16, 5, 7), gpu)
                big[:, 8:8 + t.shape[1]].copy_(t.to(gpu).to(torch.bfloat16))
                parts.append(big[:, 8:8 + t.shape[1]])
            else:
                parts.append(_nhwc(t, gpu))
        out = Fn.CatChannelsFn.apply(*parts)
        ref = torch.cat([_bf(t) for t in src], 1)
        assert torch.equal(out.float().cpu(), ref)


@pytest.mark.parametrize('case', CONV_CASES, ids=[str(i) for i in range(len(CONV_CASES))])
def test_conv_fwd_bwd(gpu, case):
    Fn, T, Conv2d = _mods()
    N, Cin, H, W, Cout, k, st, pad, bias, act, up2 = case
    torch.manual_seed(hash(str(case)) & 0xffff)
    m = Conv2d(Cin, Cout, k, st, pad, bias=bias)
    x = _bf(torch.randn(N, Cin, H, W))
    Wt = _bf(m.weight.detach())
    m.weight.data.copy_(Wt)
    m = m.to(gpu)
    xd = _nhwc(x, gpu).requires_grad_()
    y = m(xd, act=act, up2=up2)
    # reference
    xr = x.clone().requires_grad_()
    wr = Wt.clone().requires_grad_()
    br = m.bias.detach().cpu().clone().requires_grad_() if bias else None
    xin = F.interpolate(xr, scale_factor=2) if up2 else xr
    yr = F.conv2d(xin, wr, br, st, pad)
    if act == 'lrelu':
        yr = F.leaky_relu(yr, 0.2)
    elif act == 'relu':
        yr = F.relu(yr)
    elif act == 'tanh':
        yr = torch.tanh(yr)
    assert y.shape == yr.shape
    assert rel_l2(y.float().cpu(), yr) < 1e-2
    gy = _bf(torch.randn(yr.shape))
    yr.backward(gy)
    y.backward(_nhwc(gy, gpu))
    assert rel_l2(xd.grad.float().cpu(), xr.grad) < 2e-2
    assert rel_l2(m.weight.grad.cpu(), wr.grad) < 2e-2
    if bias:
        assert rel_l2(m.bias.grad.cpu(), br.grad) < 2e-2
    # a second backward accumulates into the existing .grad in place (direct
    # accumulation path of the weight / bias gradient kernels)
    wg0 = m.weight.grad.clone()
    y2 = m(xd.detach(), act=act, up2=up2)
    y2.backward(_nhwc(gy, gpu))
    assert rel_l2(m.weight.grad.cpu(), 2 * wg0.cpu()) < 1e-5


def test_conv_double_backward(gpu):
    """d/dW of ||d<y,r>/dx||^2 -- the gradient-penalty pattern (train.py:389-402)."""
    Fn, T, Conv2d = _mods()
    torch.manual_seed(3)
    for (Cin, Cout, k, st, pad) in [(8, 16, 4, 2, 1), (16, 16, 3, 1, 1), (3, 8, 3, 1, 1)]:
        m = Conv2d(Cin, Cout, k, st, pad, bias=False)
        Wt = _bf(m.weight.detach())
        m.weight.data.copy_(Wt)
        m = m.to(gpu)
        x = _bf(torch.randn(2, Cin, 8, 8))
        r = _bf(torch.randn(2, Cout, (8 + 2 * pad - k) // st + 1, (8 + 2 * pad - k) // st + 1))
        xd = _nhwc(x, gpu).requires_grad_()
        y = m(xd, act='lrelu')
        (gx,) = torch.autograd.grad(y, xd, _nhwc(r, gpu), create_graph=True)
        loss = Fn.DotFn.apply(gx, gx)
        loss.backward()
        xr = x.clone().requires_grad_()
        wr = Wt.clone().requires_grad_()
        yr = F.leaky_relu(F.conv2d(xr, wr, None, st, pad), 0.2)
        (gxr,) = torch.autograd.grad(yr, xr, r, create_graph=True)
        (gxr * gxr).sum().backward()
        assert rel_l2(loss.detach().cpu(), (gxr * gxr).sum().detach()) < 2e-2
        assert rel_l2(m.weight.grad.cpu(), wr.grad) < 3e-2


@pytest.mark.parametrize('mode,up2,act,C,HW', [(0, False, 'relu', 24, 6), (0, False, 'lrelu', 24, 6),
                                               (1, True, 'relu', 24, 6), (1, False, None, 24, 6),
                                               (0, True, None, 24, 6),
                                               # power-of-two channel groups: wave-shuffle dmask path,
                                               # odd grids for the unrolled pixel loops' tails
                                               (1, True, 'relu', 64, 13), (1, False, 'relu', 32, 29),
                                               (0, False, 'lrelu', 256, 11)])
def test_bn_modulation(gpu, mode, up2, act, C, HW):
    """SyncBN (batch stats) + affine / affine_ssa modulation + act (+ fused nearest-up)."""
    Fn, T, _ = _mods()
    from eegan_hip.nn import SyncBatchNorm2d
    torch.manual_seed(5)
    N, H, W = 3, HW, HW
    bn = SyncBatchNorm2d(C, affine=(mode == 0))
    if mode == 0:
        bn.weight.data.normal_(1, 0.2)
        bn.bias.data.normal_(0, 0.2)
    bn = bn.to(gpu)
    x = _bf(torch.randn(N, C, H, W) * 2 + 0.5)
    Ho, Wo = (2 * H, 2 * W) if up2 else (H, W)
    gam = torch.randn(N, C) * 0.5
    bet = torch.randn(N, C) * 0.5
    msk = torch.rand(N, 1, Ho, Wo)
    xd = _nhwc(x, gpu).requires_grad_()
    gd, bd, md = gam.to(gpu).requires_grad_(), bet.to(gpu).requires_grad_(), msk.to(gpu).requires_grad_()
    if mode == 0:
        y = bn(xd, act=act, up2=up2)
    else:
        y = bn.modulate(xd, gd, bd, md, act=act, up2=up2)
    xr = x.clone().requires_grad_()
    gr, br_, mr = gam.clone().requires_grad_(), bet.clone().requires_grad_(), msk.clone().requires_grad_()
    wr = bn.weight.detach().cpu().clone().requires_grad_() if mode == 0 else None
    bb = bn.bias.detach().cpu().clone().requires_grad_() if mode == 0 else None
    rm, rv = torch.zeros(C), torch.ones(C)
    xin = F.interpolate(xr, scale_factor=2) if up2 else xr
    n = F.batch_norm(xin, rm, rv, wr, bb, True, 0.1, 1e-5)
    if mode == 1:
        n = (gr[:, :, None, None] * mr + 1) * n + br_[:, :, None, None] * mr
    if act == 'relu':
        n = F.relu(n)
    elif act == 'lrelu':
        n = F.leaky_relu(n, 0.2)
    assert rel_l2(y.float().cpu(), n) < 1e-2
    assert rel_l2(bn.running_mean.cpu(), rm) < 1e-4
    assert rel_l2(bn.running_var.cpu(), rv) < 1e-4
    g = _bf(torch.randn(n.shape))
    n.backward(g)
    y.backward(_nhwc(g, gpu))
    assert rel_l2(xd.grad.float().cpu(), xr.grad) < 2e-2
    if mode == 0:
        assert rel_l2(bn.weight.grad.cpu(), wr.grad) < 1e-2
        assert rel_l2(bn.bias.grad.cpu(), bb.grad) < 1e-2
    else:
        assert rel_l2(gd.grad.cpu(), gr.grad) < 1e-2
        assert rel_l2(bd.grad.cpu(), br_.grad) < 1e-2
        assert rel_l2(md.grad.cpu(), mr.grad) < 1e-2


def test_elementwise_ops(gpu):
    Fn, T, _ = _mods()
    torch.manual_seed(7)
    x = _bf(torch.randn(2, 24, 8, 8))
    # avg pool 2 + adjoint + double adjoint
    xd = _nhwc(x, gpu).requires_grad_()
    y = Fn.AvgPool2Fn.apply(xd)
    assert rel_l2(y.float().cpu(), F.avg_pool2d(x, 2)) < 1e-2
    # upsample
    u = Fn.Upsample2Fn.apply(_nhwc(x, gpu))
    assert rel_l2(u.float().cpu(), F.interpolate(x, scale_factor=2)) < 1e-6
    # scale-add with device gamma
    h = _bf(torch.randn(2, 24, 8, 8))
    gm = torch.tensor([0.7], device=gpu)
    o = Fn.ScaleAddFn.apply(_nhwc(x, gpu), _nhwc(h, gpu), gm)
    assert rel_l2(o.float().cpu(), x + 0.7 * h) < 1e-2
    # cat + tile cond, and its adjoint
    f = _nhwc(x[:, :, :4, :4].contiguous(), gpu).requires_grad_()
    c = torch.randn(2, 256, device=gpu, requires_grad=True)
    ct = Fn.CatTileFn.apply(f, c)
    ref = torch.cat([x[:, :, :4, :4], c.detach().cpu().view(2, 256, 1, 1).repeat(1, 1, 4, 4)], 1)
    assert rel_l2(ct.float().cpu(), ref) < 1e-2
    gct = _bf(torch.randn(ref.shape))
    ct.backward(_nhwc(gct, gpu))
    assert rel_l2(c.grad.cpu(), gct[:, 24:].sum((2, 3))) < 1e-2
    assert rel_l2(f.grad.float().cpu(), gct[:, :24]) < 1e-6
    # mask bilinear (align_corners=True) + sigmoid and its backward
    m = torch.randn(2, 1, 8, 8)
    md = m.to(gpu).requires_grad_()
    s = Fn.MaskResizeSigmoidFn.apply(md, 16)
    mr = m.clone().requires_grad_()
    sr = torch.sigmoid(F.interpolate(mr, size=16, mode='bilinear', align_corners=True))
    assert rel_l2(s.cpu(), sr) < 1e-5
    gs = torch.randn(sr.shape)
    sr.backward(gs)
    s.backward(gs.to(gpu))
    assert rel_l2(md.grad.cpu(), mr.grad) < 1e-5
    # image bilinear 256 -> 299 (align_corners=False)
    im = _bf(torch.rand(2, 3, 32, 32) * 2 - 1)
    imd = _nhwc(im, gpu).requires_grad_()
    r = Fn.BilinearFn.apply(imd, 37, 37)
    imr = im.clone().requires_grad_()
    rr = F.interpolate(imr, size=(37, 37), mode='bilinear', align_corners=False)
    assert rel_l2(r.float().cpu(), rr) < 1e-2
    g2 = _bf(torch.randn(rr.shape))
    rr.backward(g2)
    r.backward(_nhwc(g2, gpu))
    assert rel_l2(imd.grad.float().cpu(), imr.grad) < 1e-2
    # gather-form adjoint over up/down ratios and both corner modes (fp32 path)
    for (hi, ho) in [(4, 64), (8, 13), (37, 16), (5, 1), (16, 16)]:
        m = torch.randn(2, 1, hi, hi)
        md = m.to(gpu).requires_grad_()
        s = Fn.MaskResizeSigmoidFn.apply(md, ho)
        mr = m.clone().requires_grad_()
        sr = torch.sigmoid(F.interpolate(mr, size=ho, mode='bilinear', align_corners=True))
        gs = torch.randn(sr.shape)
        sr.backward(gs)
        s.backward(gs.to(gpu))
        assert rel_l2(md.grad.cpu(), mr.grad) < 1e-5, (hi, ho)
    for (hi, ho) in [(37, 16), (16, 16), (7, 19), (32, 299)]:
        im = _bf(torch.rand(1, 3, hi, hi) * 2 - 1)
        imd = _nhwc(im, gpu).requires_grad_()
        r = Fn.BilinearFn.apply(imd, ho, ho)
        imr = im.clone().requires_grad_()
        rr = F.interpolate(imr, size=(ho, ho), mode='bilinear', align_corners=False)
        g2 = _bf(torch.randn(rr.shape))
        rr.backward(g2)
        r.backward(_nhwc(g2, gpu))
        assert rel_l2(imd.grad.float().cpu(), imr.grad) < 1e-2, (hi, ho)
    # max pool 3x3 s2 / avg pool 3x3 s1 p1 / global average pool
    z = _bf(torch.randn(2, 16, 11, 11))
    zd = _nhwc(z, gpu).requires_grad_()
    mp = Fn.MaxPool3s2Fn.apply(zd)
    zr = z.clone().requires_grad_()
    mpr = F.max_pool2d(zr, 3, 2)
    assert rel_l2(mp.float().cpu(), mpr) < 1e-6
    gm2 = _bf(torch.randn(mpr.shape))
    mpr.backward(gm2)
    mp.backward(_nhwc(gm2, gpu))
    assert rel_l2(zd.grad.float().cpu(), zr.grad) < 1e-2
    ap = Fn.AvgPool3s1Fn.apply(_nhwc(z, gpu))
    assert rel_l2(ap.float().cpu(), F.avg_pool2d(z, 3, 1, 1)) < 1e-2
    ga = Fn.GlobalAvgPoolFn.apply(_nhwc(z, gpu))
    assert rel_l2(ga.cpu(), z.mean((2, 3))) < 1e-3
    # fc -> NHWC view and back
    fc = torch.randn(3, 32 * 16)
    fcd = fc.to(gpu).requires_grad_()
    v = Fn.FcToNhwcFn.apply(fcd, 32)
    assert rel_l2(v.float().cpu(), fc.view(3, 32, 4, 4)) < 1e-2
    gv = _bf(torch.randn(3, 32, 4, 4))
    v.backward(_nhwc(gv, gpu))
    assert rel_l2(fcd.grad.cpu(), gv.reshape(3, -1)) < 1e-6


def test_wgrad_staged_epilogue_bit_identical(gpu, monkeypatch):
    """Unsplit weight gradients through the LDS-staged dW epilogue
    (EEGAN_CONV wgrad_stage_epi=1, default: 16-B read-add-write runs) equal the
    direct epilogue bit for bit, fresh and accumulated into an existing
    gradient; the DiscCond-head shapes (4x4 grids, 768 / 1024 channels) and
    ragged tiles (Cout, K not multiples of the tile)."""
    Fn, T, _ = _mods()
    conv_knob(monkeypatch, 'wgrad_target', '1')   # one split: the direct dW path
    for N, Cin, H, W, Cout, k, st, pad in [(8, 768, 4, 4, 1024, 3, 1, 1), (8, 1024, 4, 4, 512, 4, 4, 0),
                                            (4, 96, 8, 8, 72, 3, 1, 1), (2, 64, 16, 16, 200, 4, 2, 1),
                                            (4, 256, 8, 8, 48, 1, 1, 0)]:
        torch.manual_seed(Cin + H + Cout)
        g = Fn.Geom(Cout, k, k, st, pad, pad, 0)
        x = _nhwc(torch.randn(N, Cin, H, W), gpu)
        Ho, Wo = g.out_hw(H, W)
        dz = _nhwc(torch.randn(N, Cout, Ho, Wo), gpu)
        outs = []
        for v in ('0', '1'):
            conv_knob(monkeypatch, 'wgrad_stage_epi', v)
            dW = torch.full((Cout, Cin, k, k), 0.5, device=gpu).contiguous(memory_format=torch.channels_last)
            Fn.conv_bwd_weight_raw(x, dz, g, (Cout, Cin, k, k), out=dW)
            outs.append((Fn.conv_bwd_weight_raw(x, dz, g, (Cout, Cin, k, k)).cpu(), dW.cpu()))
        for a_, b_ in zip(*outs):
            assert torch.equal(a_, b_), (N, Cin, H, Cout, k)
        wr = torch.zeros(Cout, Cin, k, k, requires_grad=True)
        F.conv2d(x.float().cpu(), wr, None, st, pad).backward(dz.float().cpu())
        assert rel_l2(outs[1][0], wr.grad) < 1e-4


def test_wgrad_xcd_remap_bit_identical(gpu, monkeypatch):
    """Weight-gradient tiles remapped so one (co tile, split)'s k tiles share an
    XCD (EEGAN_CONV wgrad_xcd=1, default) compute the same tiles: torch.equal with
    the plain block order, split and unsplit, fresh and accumulated -- on the
    pipelined kernel for power-of-two grids and on the LDS-DMA kernel for the
    others (17^2, and up2 sources: the generator's upsampling convs)."""
    Fn, T, _ = _mods()
    for N, Cin, H, W, Cout, k, st, pad, up2 in [(16, 128, 32, 32, 128, 3, 1, 1, 0), (8, 64, 64, 64, 64, 3, 1, 1, 0),
                                                 (8, 64, 32, 32, 128, 4, 2, 1, 0), (8, 768, 4, 4, 1024, 3, 1, 1, 0),
                                                 (16, 192, 17, 17, 192, 3, 1, 1, 0), (8, 128, 16, 16, 128, 3, 1, 1, 1),
                                                 (4, 64, 32, 32, 32, 3, 1, 1, 1)]:
        torch.manual_seed(Cin + H + Cout)
        g = Fn.Geom(Cout, k, k, st, pad, pad, up2)
        x = _nhwc(torch.randn(N, Cin, H, W), gpu)
        Ho, Wo = g.out_hw(H, W)
        dz = _nhwc(torch.randn(N, Cout, Ho, Wo), gpu)
        outs = []
        for v in ('0', '1'):
            conv_knob(monkeypatch, 'wgrad_xcd', v)
            dW = torch.full((Cout, Cin, k, k), 0.25, device=gpu).contiguous(memory_format=torch.channels_last)
            Fn.conv_bwd_weight_raw(x, dz, g, (Cout, Cin, k, k), out=dW)
            outs.append((Fn.conv_bwd_weight_raw(x, dz, g, (Cout, Cin, k, k)).cpu(), dW.cpu()))
        for a_, b_ in zip(*outs):
            assert torch.equal(a_, b_), (N, Cin, H, Cout, k)


def test_wgrad_quad_slab_bit_identical(gpu, monkeypatch):
    """Split weight gradients written as co-quad slabs (EEGAN_CONV wgrad_quad=1,
    default: one 16-B store per lane) reduce to the same bits as the row-major
    slabs: the column sums visit the same splits in the same order.  Covers
    accumulation into an existing gradient and Cout % 4 != 0 (row-major)."""
    Fn, T, _ = _mods()
    conv_knob(monkeypatch, 'wgrad_quad_mink', '0')   # quad slabs at every K (default: K > 1024)
    for N, Cin, H, W, Cout, k, st, pad in [(4, 64, 32, 32, 64, 3, 1, 1), (2, 128, 16, 16, 256, 4, 2, 1),
                                            (8, 32, 64, 64, 36, 3, 1, 1), (16, 256, 8, 8, 512, 3, 1, 1)]:
        torch.manual_seed(Cin + H + Cout)
        g = Fn.Geom(Cout, k, k, st, pad, pad, 0)
        x = _nhwc(torch.randn(N, Cin, H, W), gpu)
        Ho, Wo = g.out_hw(H, W)
        dz = _nhwc(torch.randn(N, Cout, Ho, Wo), gpu)
        outs = []
        # row-major slabs with direct stores / co-quad slabs / row-major slabs through the LDS-staged epilogue
        for q, stg in (('0', '1'), ('1', '1'), ('0', '2')):
            conv_knob(monkeypatch, 'wgrad_stage_epi', stg)
            conv_knob(monkeypatch, 'wgrad_quad', q)
            dW = torch.ones(Cout, Cin, k, k, device=gpu).contiguous(memory_format=torch.channels_last)
            Fn.conv_bwd_weight_raw(x, dz, g, (Cout, Cin, k, k), out=dW)
            outs.append((Fn.conv_bwd_weight_raw(x, dz, g, (Cout, Cin, k, k)).cpu(), dW.cpu()))
        for o in outs[1:]:
            for a, b in zip(outs[0], o):
                assert torch.equal(a, b), (N, Cin, H, Cout)
        xr = x.float().cpu().requires_grad_()
        wr = torch.zeros(Cout, Cin, k, k, requires_grad=True)
        F.conv2d(x.float().cpu(), wr, None, st, pad).backward(dz.float().cpu())
        assert rel_l2(outs[1][0], wr.grad) < 1e-4


@pytest.mark.parametrize('P', [64, 4096, 1 << 18])
def test_dot_partials_finish(gpu, P):
    """<g, h> from per-block partials and the fixed-order dot_final launch:
    deterministic over repeated calls, the scale-add backward's fused <g, h>
    accumulated into a sink, against the fp64 sum of the bf16 inputs."""
    Fn, T, _ = _mods()
    torch.manual_seed(11)
    C = 40
    x = _nhwc(_bf(torch.randn(1, C, P // 64, 64)), gpu)
    y = _nhwc(_bf(torch.randn(1, C, P // 64, 64)), gpu)
    ref = (x.double() * y.double()).sum().item()
    vals = [Fn._dot_raw(x, y).item() for _ in range(3)]
    assert vals[0] == vals[1] == vals[2], vals
    g = torch.zeros(1, device=gpu)
    gm = torch.tensor([0.5], device=gpu)
    d = torch.empty_like(x)
    ws = T.workspace(Fn.ops.dot_workspace(), gpu)
    for _ in range(2):   # accumulate twice into the sink
        Fn.ops.scale_dot(x.data_ptr(), Fn.ld_of(x), y.data_ptr(), Fn.ld_of(y), gm.data_ptr(), 1.0, P, C,
                         d.data_ptr(), Fn.ld_of(d), ws.data_ptr(), g.data_ptr(), 1, 0, 0.2, Fn.stream())
    assert abs(g.item() - 2 * ref) <= 1e-5 * abs(2 * ref) + 1e-3, (g.item(), ref)
    assert rel_l2(d.float().cpu(), 0.5 * x.float().cpu()) < 1e-2
    assert abs(vals[0] - ref) <= 1e-5 * max(abs(ref), 1.0), (vals, ref)


def test_linear_and_attr(gpu):
    Fn, T, _ = _mods()
    from eegan_hip.nn import Linear
    torch.manual_seed(9)
    lin = Linear(100, 70).to(gpu)
    x = torch.randn(5, 100)
    xd = x.to(gpu).requires_grad_()
    y = lin(xd, act='relu')
    wr = lin.weight.detach().cpu().clone().requires_grad_()
    br = lin.bias.detach().cpu().clone().requires_grad_()
    xr = x.clone().requires_grad_()
    yr = F.relu(F.linear(xr, wr, br))
    assert rel_l2(y.cpu(), yr) < 1e-5
    g = torch.randn(yr.shape)
    yr.backward(g)
    y.backward(g.to(gpu))
    assert rel_l2(xd.grad.cpu(), xr.grad) < 1e-5
    assert rel_l2(lin.weight.grad.cpu(), wr.grad) < 1e-5
    assert rel_l2(lin.bias.grad.cpu(), br.grad) < 1e-5
    q, k, v = [torch.randn(3, 4, 256) for _ in range(3)]
    qd, kd, vd = [t.to(gpu).requires_grad_() for t in (q, k, v)]
    o = Fn.AttrAttnFn.apply(qd, kd, vd, 1 / 16)
    qr, kr, vr = [t.clone().requires_grad_() for t in (q, k, v)]
    orf = torch.bmm(torch.softmax(torch.bmm(qr, kr.transpose(1, 2)), -1) / 16, vr)
    assert rel_l2(o.cpu(), orf) < 1e-5
    go = torch.randn(orf.shape)
    orf.backward(go)
    o.backward(go.to(gpu))
    for a, b in [(qd, qr), (kd, kr), (vd, vr)]:
        assert rel_l2(a.grad.cpu(), b.grad) < 1e-4


def test_losses_small(gpu):
    Fn, T, _ = _mods()
    torch.manual_seed(11)
    x = torch.randn(7)
    for mode, fn in [(0, lambda t: F.relu(1 - t).mean()), (1, lambda t: F.relu(1 + t).mean()),
                     (2, lambda t: -t.mean()), (3, lambda t: t.mean())]:
        xd = x.to(gpu).requires_grad_()
        o = Fn.DoutReduceFn.apply(xd, mode)
        xr = x.clone().requires_grad_()
        orf = fn(xr)
        assert abs(o.item() - orf.item()) < 1e-5
        o.backward()
        orf.backward()
        assert rel_l2(xd.grad.cpu(), xr.grad) < 1e-5
    lg = torch.randn(4, 10)
    tg = torch.zeros(4, 10)
    tg[torch.arange(4), torch.tensor([1, 5, 9, 0])] = 1
    ld = lg.to(gpu).requires_grad_()
    o = Fn.BceLogitsFn.apply(ld, tg.to(gpu))
    lr = lg.clone().requires_grad_()
    orf = F.binary_cross_entropy_with_logits(lr, tg)
    assert abs(o.item() - orf.item()) < 1e-5
    o.backward()
    orf.backward()
    assert rel_l2(ld.grad.cpu(), lr.grad) < 1e-5
    # gradient penalty
    gx = _bf(torch.randn(3, 3, 8, 8) * 0.1)
    gs = torch.randn(3, 256) * 0.05
    gxd, gsd = _nhwc(gx, gpu).requires_grad_(), gs.to(gpu).requires_grad_()
    o = Fn.GradPenaltyFn.apply(gxd, gsd)
    gxr, gsr = gx.clone().requires_grad_(), gs.clone().requires_grad_()
    g = torch.cat([gxr.reshape(3, -1), gsr], 1)
    orf = 2.0 * torch.mean(torch.sqrt((g ** 2).sum(1)) ** 6)
    assert abs(o.item() - orf.item()) / orf.item() < 1e-4
    o.backward()
    orf.backward()
    assert rel_l2(gxd.grad.float().cpu(), gxr.grad) < 1e-2
    assert rel_l2(gsd.grad.cpu(), gsr.grad) < 1e-4


def test_class_onehot_bit_exact(gpu):
    Fn, T, _ = _mods()
    from oracle import eegan_oracle as O
    ids = torch.tensor([1, 200, 0, 57, 57, 3])
    got, err = Fn.class_onehot(ids, 6, 200, gpu)
    assert torch.equal(got.cpu(), O.prepare_class_labels(6, 200, ids.tolist()))
    assert err.item() == 0


@pytest.mark.parametrize('beta1', [0.0, 0.5])
def test_adam_matches_torch(gpu, beta1):
    """beta1 = 0 (train.py's betas) takes the kernel form that does not read
    the old first moment; 0.5 the general lerp."""
    from eegan_hip.optim import FlatAdam
    torch.manual_seed(13)
    # (1000, 3001): several grid-stride groups per thread and a ragged float4 tail
    ps = [torch.nn.Parameter(torch.randn(s, device=gpu)) for s in [(7, 3), (5,), (1,), (33, 2, 3), (1000, 3001)]]
    qs = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    opt = FlatAdam(ps, lr=4e-4, betas=(beta1, 0.9))
    ref = torch.optim.Adam(qs, lr=4e-4, betas=(beta1, 0.9))
    for it in range(3):
        gs = [torch.randn(p.shape, device=gpu) for p in ps]
        opt.zero_grad()
        ref.zero_grad()
        for p, q, g in zip(ps, qs, gs):
            p.grad.add_(g)
            q.grad = g.clone()
        opt.step()
        ref.step()
    for p, q in zip(ps, qs):
        assert torch.allclose(p.detach(), q.detach(), rtol=1e-5, atol=1e-7)


def test_flat_adam_repacks_conv_weights(gpu):
    """After FlatAdam.step() every registered conv weight pack (forward and
    bwd-data image, refreshed by ONE batched launch) equals a fresh per-weight
    pack of the updated weights, and the caches are marked current."""
    from eegan_hip.optim import FlatAdam
    Fn, T, Conv2d = _mods()
    torch.manual_seed(21)
    m1 = Conv2d(3, 40, 3, 1, 1).to(gpu)
    m2 = Conv2d(40, 136, 4, 2, 1).to(gpu)
    m3 = Conv2d(136, 3, 1, 1, 0).to(gpu)
    m4 = Conv2d(3, 192, 1, 1, 0).to(gpu)      # 192 output channels: three 64-wide bwd-image column tiles
    m5 = Conv2d(256, 160, 4, 2, 1).to(gpu)    # 16-byte forward-image loads, multi-tile bwd image, 16 taps
    mods = (m1, m2, m3, m4, m5)
    opt = FlatAdam([p for m in mods for p in m.parameters()], lr=1e-2, betas=(0.0, 0.9))
    for _ in range(2):
        opt.zero_grad()
        x = _nhwc(_bf(torch.randn(2, 3, 8, 8)), gpu).requires_grad_()
        y = m3(m2(m1(x, act='lrelu')))
        z = m5(_nhwc(_bf(torch.randn(2, 256, 8, 8)), gpu).requires_grad_())
        u = m4(x)
        (y.float().sum() + z.float().sum() + u.float().sum()).backward()
        opt.step()
    for m in mods:
        c = m._cache
        assert c.fwd is not None and c.bwd is not None
        for tr, buf, key in ((False, c.fwd, c.fwd_key), (True, c.bwd, c.bwd_key)):
            assert key == Fn.PackCache._key(m.weight)
            assert torch.equal(buf, Fn.pack_weight(m.weight, tr))


def test_flat_adam_fused_pack_bit_identical(gpu, monkeypatch):
    """eegan_adam_pack (the Adam step fused with the conv weight re-pack, one
    launch; optim.ADAM_PACK, default) against eegan_adam + the batched pack:
    parameters, both Adam moments and every pack torch.equal after two steps
    -- conv weights with 3 / 1 / 192 / 1024 channels (ragged 64-wide tiles,
    Cgp 8 runs), 4x4 / 3x3 / 1x1 taps, biases and alignment gaps as range jobs."""
    from eegan_hip import optim
    Fn, T, Conv2d = _mods()
    runs = []
    for fused in (False, True):
        torch.manual_seed(33)
        mods = (Conv2d(3, 40, 3, 1, 1).to(gpu), Conv2d(40, 136, 4, 2, 1).to(gpu), Conv2d(136, 1, 1, 1, 0).to(gpu),
                Conv2d(3, 192, 1, 1, 0).to(gpu), Conv2d(136, 1024, 3, 1, 1, bias=False).to(gpu))
        extra = torch.nn.Parameter(torch.randn(7, device=gpu))    # a non-conv parameter (range job, gap after it)
        opt = optim.FlatAdam([p for m in mods for p in m.parameters()] + [extra], lr=1e-2, betas=(0.0, 0.9))
        monkeypatch.setattr(optim, 'ADAM_PACK', fused)
        torch.manual_seed(34)
        for _ in range(2):
            opt.zero_grad()
            x = _nhwc(_bf(torch.randn(2, 3, 8, 8)), gpu).requires_grad_()
            h = mods[1](mods[0](x, act='lrelu'))
            y = mods[2](h)
            u = mods[3](x)
            w = mods[4](h)
            (y.float().sum() + u.float().sum() + w.float().square().mean() + (extra * extra).sum()).backward()
            opt.step()
        torch.cuda.synchronize()
        runs.append((opt.flat.clone(), opt.m.clone(), opt.v.clone(),
                     [(m._cache.fwd.clone(), m._cache.bwd.clone()) for m in mods]))
        for m in mods:
            for tr, buf in ((False, m._cache.fwd), (True, m._cache.bwd)):
                assert torch.equal(buf, Fn.pack_weight(m.weight, tr)), (fused, tr, tuple(m.weight.shape))
    (p0, m0, v0, k0), (p1, m1, v1, k1) = runs
    assert torch.equal(p0, p1) and torch.equal(m0, m1) and torch.equal(v0, v1)
    for (f0, b0), (f1, b1) in zip(k0, k1):
        assert torch.equal(f0, f1) and torch.equal(b0, b1)


@pytest.mark.parametrize('th', ['16', '8', '0'])
def test_conv_halo3_matches_tile_kernel(gpu, monkeypatch, th):
    """3x3 / stride-1 convs on the LDS halo-tile kernel (conv_halo3_kernel,
    EEGAN_CONV halo=1, default) against the tile kernels (halo=0) and torch's
    fp32 conv: forward with bias / act / residual + gain and the fused nearest-2x
    upsample, backward-data plain / gated / with the half-resolution residual;
    ragged input channels (40 -> a masked chunk), two output-channel tiles with a
    partial second one (96), 32 output channels (half a tile), both tile heights
    double-buffered (halo_th 16 / 8) and the default single-buffered 4-row form
    that runs three workgroups per CU (halo_th 0).  The halo kernel sums slice-major
    (the tile kernels tap-major), so the gate is bf16 output rounding: rel-L2
    <= 5e-3 between the kernels, <= 1e-2 against fp32."""
    Fn, T, _ = _mods()
    conv_knob(monkeypatch, 'halo_th', th)
    lrelu = Fn.ACT_CODES['lrelu']
    for N, Cin, H, W, Cout, up2 in [(2, 64, 32, 64, 64, 0), (3, 40, 16, 32, 96, 0), (2, 128, 16, 32, 48, 0),
                                    (2, 64, 16, 32, 64, 1), (1, 256, 32, 32, 128, 0), (2, 64, 16, 32, 32, 0)]:
        torch.manual_seed(N * Cin + Cout + H + up2)
        g = Fn.Geom(Cout, 3, 3, 1, 1, 1, up2)
        xs = torch.randn(N, Cin, H // 2, W // 2) if up2 else torch.randn(N, Cin, H, W)
        x = _nhwc(xs, gpu)
        Wt = (torch.randn(Cout, Cin, 3, 3) * (1.0 / (9 * Cin) ** 0.5)).to(gpu)
        b = torch.randn(Cout).to(gpu) * 0.1
        gam = torch.tensor([0.7]).to(gpu)
        res = _nhwc(torch.randn(N, Cout, H, W), gpu)
        dz = _nhwc(torch.randn(N, Cout, H, W), gpu)
        gate = _nhwc(torch.randn(N, Cin, H, W), gpu)
        halfres = _nhwc(torch.randn(N, Cin, H // 2, W // 2), gpu)
        outs = {}
        for on in ('0', '1'):
            conv_knob(monkeypatch, 'halo', on)
            o = [Fn.conv_fwd_raw(x, Wt, b, g, act=lrelu, res=res, gamma=gam).float().cpu(),
                 Fn.conv_fwd_raw(x, Wt, None, g).float().cpu()]
            if not up2:
                o += [Fn.conv_bwd_data_raw(dz, Wt, g, tuple(x.shape)).float().cpu(),
                      Fn.conv_bwd_data_raw(dz, Wt, g, tuple(x.shape), gate=gate, gate_act=lrelu).float().cpu(),
                      Fn.conv_bwd_data_raw(dz, Wt, g, tuple(x.shape), res=halfres, res_up2=1,
                                           res_scale=0.25).float().cpu()]
            outs[on] = o
        for k, (a, c) in enumerate(zip(outs['1'], outs['0'])):
            e = rel_l2(a, c)
            assert e <= 5e-3, (N, Cin, H, W, Cout, up2, k, e)
        xin = xs.to(torch.bfloat16).float()
        if up2:
            xin = F.interpolate(xin, scale_factor=2, mode='nearest')
        ref = F.conv2d(xin, Wt.cpu().to(torch.bfloat16).float(), None, 1, 1)
        assert rel_l2(outs['1'][1], ref) <= 1e-2
        if not up2:
            dref = F.conv_transpose2d(dz.float().cpu(), Wt.cpu().to(torch.bfloat16).float(), None, 1, 1)
            assert rel_l2(outs['1'][2], dref) <= 1e-2


@pytest.mark.gpu
@pytest.mark.parametrize('tpb', [0, 1, 3, 7])
def test_conv_halo3r_matches_halo3(gpu, monkeypatch, tpb):
    """64-channel 3x3 convs on the resident-weight halo kernel (conv_halo3r_kernel,
    EEGAN_CONV halo_r=1, default) against conv_halo3_kernel (halo_r=0): the same
    K order, so the same bits -- forward with bias / act / residual + gain, the
    fused nearest-2x upsample, backward-data plain / gated / with the half-
    resolution residual; two output-channel tiles (128), and tiles per workgroup
    auto / 1 / 3 / 7 (ragged last workgroups, tile walks crossing image rows and
    images)."""
    Fn, T, _ = _mods()
    conv_knob(monkeypatch, 'halo_r_tpb', tpb)
    lrelu = Fn.ACT_CODES['lrelu']
    for N, Cin, H, W, Cout, up2 in [(2, 64, 32, 64, 64, 0), (2, 64, 16, 32, 128, 0), (3, 64, 16, 64, 64, 1),
                                    (5, 64, 8, 32, 64, 0), (2, 128, 16, 32, 64, 0)]:
        torch.manual_seed(N * Cin + Cout + H + up2)
        g = Fn.Geom(Cout, 3, 3, 1, 1, 1, up2)
        xs = torch.randn(N, Cin, H // 2, W // 2) if up2 else torch.randn(N, Cin, H, W)
        x = _nhwc(xs, gpu)
        Wt = (torch.randn(Cout, Cin, 3, 3) * (1.0 / (9 * Cin) ** 0.5)).to(gpu)
        b = torch.randn(Cout).to(gpu) * 0.1
        gam = torch.tensor([0.7]).to(gpu)
        res = _nhwc(torch.randn(N, Cout, H, W), gpu)
        dz = _nhwc(torch.randn(N, Cout, H, W), gpu)
        gate = _nhwc(torch.randn(N, Cin, H, W), gpu)
        halfres = _nhwc(torch.randn(N, Cin, H // 2, W // 2), gpu)
        outs = {}
        for on in ('0', '1'):
            conv_knob(monkeypatch, 'halo_r', on)
            o = [Fn.conv_fwd_raw(x, Wt, b, g, act=lrelu, res=res, gamma=gam).float().cpu(),
                 Fn.conv_fwd_raw(x, Wt, None, g).float().cpu()]
            if not up2:
                o += [Fn.conv_bwd_data_raw(dz, Wt, g, tuple(x.shape)).float().cpu(),
                      Fn.conv_bwd_data_raw(dz, Wt, g, tuple(x.shape), gate=gate, gate_act=lrelu).float().cpu(),
                      Fn.conv_bwd_data_raw(dz, Wt, g, tuple(x.shape), res=halfres, res_up2=1,
                                           res_scale=0.25).float().cpu()]
            outs[on] = o
        for k, (a, c) in enumerate(zip(outs['1'], outs['0'])):
            assert torch.equal(a, c), (N, Cin, H, W, Cout, up2, k, float((a - c).abs().max()))
        xin = xs.to(torch.bfloat16).float()
        if up2:
            xin = F.interpolate(xin, scale_factor=2, mode='nearest')
        ref = F.conv2d(xin, Wt.cpu().to(torch.bfloat16).float(), None, 1, 1)
        assert rel_l2(outs['1'][1], ref) <= 1e-2


@pytest.mark.gpu
def test_conv_halo3_ragged_channels(gpu, monkeypatch):
    """The halo kernel on get_mask's 100-channel conv (models.py:34-41): the
    forward's 100 output rows end in a partial 8-channel chunk (its valid
    channels stored one by one, nothing past 100 written), the data gradient
    reads a 100-channel dy whose padding channels hold NaN bits (masked in the
    B fragments).  Against the tile kernels (halo=0) and torch fp32."""
    Fn, T, _ = _mods()
    N, Cin, H, W, Cout = 2, 64, 16, 32, 100
    torch.manual_seed(7)
    g = Fn.Geom(Cout, 3, 3, 1, 1, 1, 0)
    xs = torch.randn(N, Cin, H, W)
    x = _nhwc(xs, gpu)
    Wt = (torch.randn(Cout, Cin, 3, 3) * (1.0 / (9 * Cin) ** 0.5)).to(gpu)
    b = torch.randn(Cout).to(gpu) * 0.1
    dzs = torch.randn(N, Cout, H, W)
    dz = _nhwc_nan_padded(dzs, gpu)
    outs = {}
    for on in ('0', '1'):
        conv_knob(monkeypatch, 'halo', on)
        y = Fn.conv_fwd_raw(x, Wt, b, g, act=Fn.ACT_CODES['relu'])
        dx = Fn.conv_bwd_data_raw(dz, Wt, g, tuple(x.shape))
        outs[on] = (y.float().cpu(), dx.float().cpu())
    for a, c in zip(outs['1'], outs['0']):
        assert torch.isfinite(a).all()
        assert rel_l2(a, c) <= 5e-3
    wb = Wt.cpu().to(torch.bfloat16).float()
    yref = F.relu(F.conv2d(xs.to(torch.bfloat16).float(), wb, b.cpu(), 1, 1))
    assert rel_l2(outs['1'][0], yref) <= 1e-2
    dref = F.conv_transpose2d(dzs.to(torch.bfloat16).float(), wb, None, 1, 1)
    assert rel_l2(outs['1'][1], dref) <= 1e-2


@pytest.mark.gpu
def test_conv_s2fwd_matches_tile_kernel(gpu, monkeypatch):
    """4x4 / stride-2 / pad-1 forward convs with 32 input and 64 output channels
    on conv_s2fwd_kernel (resD conv_r[0] of each D's first block, models.py:267):
    the same K order as the tile kernels, so bit-identical to them (EEGAN_CONV
    s2f=0), and against torch's fp32 conv; a grid with more tiles than the
    persistent workgroups (each walks several), bias + leaky ReLU."""
    Fn, T, _ = _mods()
    lrelu = Fn.ACT_CODES['lrelu']
    for N, H, W in [(2, 32, 64), (16, 128, 128)]:
        torch.manual_seed(N + H)
        g = Fn.Geom(64, 4, 4, 2, 1, 1, 0)
        xs = torch.randn(N, 32, H, W)
        x = _nhwc(xs, gpu)
        Wt = (torch.randn(64, 32, 4, 4) * (1.0 / (16 * 32) ** 0.5)).to(gpu)
        b = torch.randn(64).to(gpu) * 0.1
        outs = {}
        for on in ('0', '1'):
            conv_knob(monkeypatch, 's2f', on)
            outs[on] = (Fn.conv_fwd_raw(x, Wt, b, g, act=lrelu).float().cpu(),
                        Fn.conv_fwd_raw(x, Wt, None, g).float().cpu())
        for a, c in zip(outs['1'], outs['0']):
            assert torch.equal(a, c), (N, H, W, float((a - c).abs().max()))
        ref = F.conv2d(xs.to(torch.bfloat16).float(), Wt.cpu().to(torch.bfloat16).float(), None, 2, 1)
        assert rel_l2(outs['1'][1], ref) <= 1e-2


@pytest.mark.parametrize('xcd', ['1', '3'])
@pytest.mark.parametrize('target', ['512', '4096'])
def test_conv_xcd_raster_bit_identical(gpu, monkeypatch, xcd, target):
    """The tile kernel's XCD raster (EEGAN_CONV xcd=1 default: G from the
    tile shape; xcd=3: three co-tile rows per group) against the plain 3-D
    grid (xcd=0): the same tiles and K order, only the block -> tile map
    differs, so torch.equal -- including grids that are not a multiple of 8
    (blocks past the grid exit), co-tile counts not divisible by the group
    height, split-K (target 4096) and the stride-2 parity classes."""
    Fn, T, _ = _mods()
    conv_knob(monkeypatch, 'target', target)
    conv_knob(monkeypatch, 'mink', '2')
    conv_knob(monkeypatch, 'xcd_minb', '1')
    lrelu = Fn.ACT_CODES['lrelu']
    for N, Cin, H, W, Cout, k, st, pad in [(2, 64, 16, 16, 128, 3, 1, 1), (3, 128, 9, 11, 320, 3, 1, 1),
                                            (2, 96, 16, 16, 256, 4, 2, 1), (16, 768, 17, 17, 192, 1, 1, 0),
                                            (4, 256, 8, 8, 512, 3, 1, 1), (5, 128, 7, 7, 200, 1, 1, 0)]:
        torch.manual_seed(N * Cin + Cout + H)
        g = Fn.Geom(Cout, k, k, st, pad, pad, 0)
        x = _nhwc(torch.randn(N, Cin, H, W), gpu)
        Wt = (torch.randn(Cout, Cin, k, k) * 0.05).to(gpu)
        b = torch.randn(Cout).to(gpu)
        gam = torch.tensor([0.7]).to(gpu)
        Ho, Wo = g.out_hw(H, W)
        res = _nhwc(torch.randn(N, Cout, Ho, Wo), gpu)
        dz = _nhwc(torch.randn(N, Cout, Ho, Wo), gpu)
        gate = _nhwc(torch.randn(N, Cin, H, W), gpu)
        outs = []
        for v in ('0', xcd):
            conv_knob(monkeypatch, 'xcd', v)
            outs.append([Fn.conv_fwd_raw(x, Wt, b, g, act=lrelu, res=res, gamma=gam).float().cpu(),
                         Fn.conv_fwd_raw(x, Wt, b, g, act=lrelu, out_f32=True).cpu(),
                         Fn.conv_bwd_data_raw(dz, Wt, g, tuple(x.shape), gate=gate, gate_act=lrelu).float().cpu()])
        for a, c in zip(*outs):
            assert torch.equal(a, c), (N, Cin, H, W, Cout, k, st, xcd, target)


def test_conv_throughput_plan(gpu, monkeypatch):
    """eegan_conv_desc.plan = 1 (a stream registered in Fn.STREAM_PLAN, as the
    trainer's TP_LANES are): the planner takes a 128-workgroup grid target --
    on these small grids fewer K splits than the latency plan -- and the
    forward, data and weight gradients still match torch fp32 (only the
    split-K summation order differs from the latency plan)."""
    Fn, T, _ = _mods()
    lane = torch.cuda.Stream()
    for N, Cin, H, W, Cout, k, st, pad in [(16, 768, 17, 17, 192, 1, 1, 0), (16, 160, 17, 17, 160, 7, 1, 3),
                                            (4, 512, 8, 8, 512, 4, 2, 1), (16, 1280, 8, 8, 320, 1, 1, 0)]:
        torch.manual_seed(N + Cin + Cout)
        kh, kw = (1, k) if k == 7 else (k, k)
        ph, pw = (0, pad) if k == 7 else (pad, pad)
        g = Fn.Geom(Cout, kh, kw, st, ph, pw, 0)
        xf = _bf(torch.randn(N, Cin, H, W))
        Wf = _bf(torch.randn(Cout, Cin, kh, kw) * (2.0 / (Cin * kh * kw)) ** 0.5)
        ref = F.conv2d(xf, Wf, stride=st, padding=(ph, pw))
        dzf = _bf(torch.randn_like(ref))
        xr = xf.clone().requires_grad_(True)
        Wr = Wf.clone().requires_grad_(True)
        F.conv2d(xr, Wr, stride=st, padding=(ph, pw)).backward(dzf)
        x = _nhwc(xf, gpu)
        Wt = Wf.to(gpu).contiguous(memory_format=torch.channels_last)
        dz = _nhwc(dzf, gpu)
        res = {}
        for plan in (0, 1):
            lane.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(lane):
                if plan:
                    Fn.STREAM_PLAN[lane.cuda_stream] = 1
                try:
                    y = Fn.conv_fwd_raw(x, Wt, None, g).float().cpu()
                    dx = Fn.conv_bwd_data_raw(dz, Wt, g, tuple(x.shape)).float().cpu()
                    dW = Fn.conv_bwd_weight_raw(x, dz, g, tuple(Wf.shape)).float().cpu()
                finally:
                    Fn.STREAM_PLAN.pop(lane.cuda_stream, None)
            torch.cuda.current_stream().wait_stream(lane)
            torch.cuda.synchronize()
            res[plan] = (y, dx, dW)
            for got, want, name in ((y, ref, 'y'), (dx, xr.grad, 'dx'), (dW, Wr.grad, 'dW')):
                e = rel_l2(got, want)
                assert e < 1e-2, (plan, name, N, Cin, Cout, k, e)
        print('throughput plan: fwd max |plan1 - plan0| %.3g' % float((res[1][0] - res[0][0]).abs().max()))
