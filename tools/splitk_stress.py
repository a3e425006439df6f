#!/usr/bin/env python
"""Stress the in-kernel split-K finish (csrc/conv.hip splitk_fused_finish) for
stale hand-offs: split-K forward / backward-data launches of several shapes on
three streams at once, beside a memory-heavy background stream, every output
compared bit for bit with the two-launch reduce (EEGAN_CONV splitk_fused=0) of
the same operands.  Prints the mismatch count per shape.

    python tools/splitk_stress.py [--iters 200]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'ee-gan_amd'))
sys.path.insert(0, REPO)
os.environ.setdefault('EEGAN_AUTO_DIST', '0')
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=200)
    args = ap.parse_args()
    from eegan_hip import functional as Fn
    from eegan_hip import tensor as T
    dev = torch.device('cuda', 0)
    lrelu = Fn.ACT_CODES['lrelu']
    shapes = [(16, 512, 4, 4, 512, 3, 1, 1), (16, 256, 8, 8, 256, 3, 1, 1), (32, 512, 8, 8, 512, 4, 2, 1),
              (32, 512, 16, 16, 512, 3, 1, 1), (16, 768, 4, 4, 1024, 3, 1, 1), (2, 96, 8, 8, 64, 4, 2, 1)]
    cases = []
    for N, Cin, H, W, Cout, k, st, pad in shapes:
        torch.manual_seed(N + Cin + Cout)
        g = Fn.Geom(Cout, k, k, st, pad, pad, 0)
        x = T.empty_nhwc(N, Cin, H, W, dev)
        x.copy_(torch.randn(N, Cin, H, W, device=dev).to(torch.bfloat16))
        Wt = torch.randn(Cout, Cin, k, k, device=dev) * 0.05
        b = torch.randn(Cout, device=dev)
        Ho, Wo = g.out_hw(H, W)
        dz = T.empty_nhwc(N, Cout, Ho, Wo, dev)
        dz.copy_(torch.randn(N, Cout, Ho, Wo, device=dev).to(torch.bfloat16))
        cases.append((g, x, Wt, b, dz))

    def run(c):
        g, x, Wt, b, dz = c
        return (Fn.conv_fwd_raw(x, Wt, b, g, act=lrelu), Fn.conv_bwd_data_raw(dz, Wt, g, tuple(x.shape)))

    os.environ['EEGAN_CONV'] = 'splitk_fused=0'
    refs = [tuple(t.clone() for t in run(c)) for c in cases]
    torch.cuda.synchronize()
    os.environ['EEGAN_CONV'] = 'splitk_fused=1'
    streams = [torch.cuda.Stream() for _ in range(3)]
    bg = torch.cuda.Stream()
    big = torch.randn(64 << 20, device=dev)
    bad = [0] * len(cases)
    outs = []
    for it in range(args.iters):
        with torch.cuda.stream(bg):
            big.mul_(1.0000001)
        for si, s in enumerate(streams):
            with torch.cuda.stream(s):
                ci = (it + si * 2) % len(cases)
                outs.append((ci, run(cases[ci])))
        if len(outs) >= 48:
            torch.cuda.synchronize()
            for ci, (y, dx) in outs:
                if not (torch.equal(y, refs[ci][0]) and torch.equal(dx, refs[ci][1])):
                    bad[ci] += 1
            outs = []
    torch.cuda.synchronize()
    for ci, (y, dx) in outs:
        if not (torch.equal(y, refs[ci][0]) and torch.equal(dx, refs[ci][1])):
            bad[ci] += 1
    left = sum(int(t.abs().sum()) for t in Fn._SPLITK_CTR.values())
    for ci, (sh, nb) in enumerate(zip(shapes, bad)):
        print('splitk stress %-40s mismatches %d' % (sh, nb))
    print('splitk stress total mismatches %d over %d launches pairs; counters left nonzero: %d'
          % (sum(bad), args.iters * len(streams), left))


if __name__ == '__main__':
    main()
