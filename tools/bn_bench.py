#!/usr/bin/env python
"""SyncBN + affine_ssa modulation kernels at the generator's large layers:
HIP-event time of the backward's reduce pass (eegan_bnmod_bwd: reduce + column
sums + per-sample sums) and dx pass (eegan_bnmod_bwd_dx) and of the forward
(statistics + fused finalize / apply), per shape.

    python tools/bn_bench.py [--iters 50]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'ee-gan_amd'))
os.environ.setdefault('EEGAN_AUTO_DIST', '0')
import torch  # noqa: E402

SHAPES = [  # N, C, H, W (physical input), up2  -- models.py SAGB affine1 / affine2 at 128^2 / 256^2
    (16, 64, 128, 128, 1), (16, 32, 256, 256, 0), (16, 64, 128, 128, 0), (16, 128, 64, 64, 1), (16, 128, 64, 64, 0),
]


def timeit(fn, iters):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=50)
    args = ap.parse_args()
    from eegan_hip import functional as Fn
    from eegan_hip._lib import ops, BnModDesc
    from eegan_hip.tensor import empty_nhwc, ld_of, stream
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    for N, C, H, W, up2 in SHAPES:
        Ho, Wo = (2 * H, 2 * W) if up2 else (H, W)
        x = Fn.to_nhwc_bf16(torch.randn(N, C, H, W, device=dev))
        g = Fn.to_nhwc_bf16(torch.randn(N, C, Ho, Wo, device=dev))
        gam = torch.randn(N, C, device=dev) * 0.1
        bet = torch.randn(N, C, device=dev) * 0.1
        mask = torch.rand(N, 1, Ho, Wo, device=dev)
        bn = torch.nn.BatchNorm2d(C, affine=False).to(dev)
        y = Fn.BnModFn.apply(x, None, None, gam, bet, mask, bn, 1, 1, 0.2, up2)
        stats = torch.empty(3 * C, device=dev)
        stats[:C] = 0.0
        stats[C:2 * C] = 1.0
        stats[2 * C:] = 1.0
        d = BnModDesc(x.data_ptr(), N, H, W, C, ld_of(x), int(up2), stats.data_ptr(), 1, 0, 0, gam.data_ptr(),
                      bet.data_ptr(), mask.data_ptr(), 1, 0.2)
        ws = torch.empty(ops.bnmod_bwd_workspace(d) // 4 + 16, device=dev)
        d0 = torch.empty(N, C, device=dev)
        d1 = torch.empty(N, C, device=dev)
        dmask = torch.empty(N, 1, Ho, Wo, device=dev)
        chan = torch.empty(2 * C, dtype=torch.float64, device=dev)
        dx = empty_nhwc(N, C, H, W, dev)
        count = float(N * Ho * Wo)
        t_red = timeit(lambda: ops.bnmod_bwd(d, g.data_ptr(), ld_of(g), ws.data_ptr(), d0.data_ptr(), d1.data_ptr(),
                                             dmask.data_ptr(), chan.data_ptr(), stream()), args.iters)
        t_dx = timeit(lambda: ops.bnmod_bwd_dx(d, g.data_ptr(), ld_of(g), chan.data_ptr(), count, dx.data_ptr(),
                                               ld_of(dx), stream()), args.iters)
        t_fwd = timeit(lambda: Fn.BnModFn.apply(x, None, None, gam, bet, mask, bn, 1, 1, 0.2, up2), args.iters)
        mb_red = (N * H * W * C * 2 + N * Ho * Wo * (C * 2 + 8)) / 1e6
        mb_dx = (N * H * W * C * 4 + N * Ho * Wo * (C * 2 + 4)) / 1e6
        print('%-22s bwd reduce %7.2f us (%5.2f TB/s)  bwd dx %7.2f us (%5.2f TB/s)  fwd %7.2f us' % (
            (N, C, H, W, up2), t_red, mb_red / t_red, t_dx, mb_dx / t_dx, t_fwd), flush=True)
        del y


if __name__ == '__main__':
    main()
