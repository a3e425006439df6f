#!/usr/bin/env python
"""Standalone conv micro-benchmark: time forward / backward-data / weight-
gradient launches of chosen bench shapes (HIP events, many back-to-back
launches), so kernel changes can be measured shape by shape.

    python tools/conv_bench.py [--shapes all|NAME,...] [--iters 50] [--dirs fwd,bwdd,wgrad]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'ee-gan_amd'))
sys.path.insert(0, REPO)

import torch  # noqa: E402

# name: (N, C, H, W, K, R, stride, pad)
SHAPES = {
    'c3x3_64_128': (16, 64, 128, 128, 64, 3, 1, 1),
    'c3x3_128_64': (16, 128, 64, 64, 128, 3, 1, 1),
    'c3x3_256_32': (16, 256, 32, 32, 256, 3, 1, 1),
    'c3x3_512_16': (16, 512, 16, 16, 512, 3, 1, 1),
    'c3x3_32_256': (16, 32, 256, 256, 32, 3, 1, 1),
    'c4x4s2_32_256': (16, 32, 256, 256, 64, 4, 2, 1),
    'c4x4s2_128_64': (16, 128, 64, 64, 256, 4, 2, 1),
    'c4x4s2_64_128': (16, 64, 128, 128, 128, 4, 2, 1),
    'c3x3_768_4': (16, 768, 4, 4, 1024, 3, 1, 1),
    'c3x3_512_4': (16, 512, 4, 4, 512, 3, 1, 1),
    'c4x4s4_1024_4': (16, 1024, 4, 4, 1024, 4, 4, 0),
    'c3x3_256_8': (16, 256, 8, 8, 256, 3, 1, 1),
    'c1x1_32_256': (16, 32, 256, 256, 64, 1, 1, 0),
    'c3x3_3_256': (16, 3, 256, 256, 32, 3, 1, 1),
    'c3x3_1024_4': (16, 768, 4, 4, 1024, 3, 1, 1),
    'c4x4s2_512_8': (16, 512, 8, 8, 512, 4, 2, 1),
    'c3x3_512_8': (16, 512, 8, 8, 512, 3, 1, 1),
    'c1x1_768_17': (16, 768, 17, 17, 192, 1, 1, 0),
    'stem_3_256x32': (32, 3, 256, 256, 32, 3, 1, 1),
    'img_32_256': (16, 32, 256, 256, 3, 3, 1, 1),
    'c3x3_32_128': (16, 32, 128, 128, 32, 3, 1, 1),
    'c1x1_32_128': (16, 32, 128, 128, 64, 1, 1, 0),
    'c1x1_64_64': (16, 64, 64, 64, 128, 1, 1, 0),
    'c1x1_128_32': (16, 128, 32, 32, 256, 1, 1, 0),
    'c1x1_256_4': (16, 256, 4, 4, 512, 1, 1, 0),
    'c1x1_100_128': (16, 100, 128, 128, 1, 1, 1, 0),
    'c3x3_64_100_128': (16, 64, 128, 128, 100, 3, 1, 1),
    'c3x3_128_100_64': (16, 128, 64, 64, 100, 3, 1, 1),
    'c3x3_64_32_128': (16, 64, 128, 128, 32, 3, 1, 1),
    'c3x3_32_16_256': (16, 32, 256, 256, 16, 3, 1, 1),
    'c3x3_64_32_256': (16, 64, 256, 256, 32, 3, 1, 1),
    # Dis256 at N = 32 (real + fake batched), models.py resD blocks 0-5
    'd256_b0_s2': (32, 32, 256, 256, 64, 4, 2, 1),
    'd256_b0_3x3': (32, 64, 128, 128, 64, 3, 1, 1),
    'd256_b1_s2': (32, 64, 128, 128, 128, 4, 2, 1),
    'd256_b1_3x3': (32, 128, 64, 64, 128, 3, 1, 1),
    'd256_b2_s2': (32, 128, 64, 64, 256, 4, 2, 1),
    'd256_b2_3x3': (32, 256, 32, 32, 256, 3, 1, 1),
    'd256_b3_s2': (32, 256, 32, 32, 512, 4, 2, 1),
    'd256_b3_3x3': (32, 512, 16, 16, 512, 3, 1, 1),
    'd256_b4_s2': (32, 512, 16, 16, 512, 4, 2, 1),
    'd256_b4_3x3': (32, 512, 8, 8, 512, 3, 1, 1),
    'd256_b5_s2': (32, 512, 8, 8, 512, 4, 2, 1),
    'd256_b5_3x3': (32, 512, 4, 4, 512, 3, 1, 1),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--shapes', default='all')
    ap.add_argument('--dirs', default='fwd,bwdd,wgrad')
    ap.add_argument('--iters', type=int, default=50)
    ap.add_argument('--device-time', action='store_true',
                    help='sum of per-dispatch HIP event times (kernel + split-K reduce), no host gaps')
    args = ap.parse_args()
    from eegan_hip import functional as Fn
    from eegan_hip.tensor import empty_nhwc
    dev = torch.device('cuda', 0)
    names = list(SHAPES) if args.shapes == 'all' else args.shapes.split(',')
    dirs = args.dirs.split(',')
    torch.manual_seed(0)
    for name in names:
        N, C, H, W, K, R, st, pd = SHAPES[name]
        g = Fn.Geom(K, R, R, st, pd, pd, 0)
        Ho, Wo = g.out_hw(H, W)
        x = empty_nhwc(N, C, H, W, dev)
        x.copy_(torch.randn(N, C, H, W, device=dev))
        dz = empty_nhwc(N, K, Ho, Wo, dev)
        dz.copy_(torch.randn(N, K, Ho, Wo, device=dev))
        Wt = (torch.randn(K, C, R, R, device=dev) * 0.05)
        dW = torch.zeros_like(Wt).contiguous(memory_format=torch.channels_last)
        cache = Fn.PackCache()
        flops = 2.0 * N * Ho * Wo * K * C * R * R
        fns = {
            'fwd': lambda: Fn.conv_fwd_raw(x, Wt, None, g, cache=cache),
            'bwdd': lambda: Fn.conv_bwd_data_raw(dz, Wt, g, tuple(x.shape), cache=cache),
            'wgrad': lambda: Fn.conv_bwd_weight_raw(x, dz, g, Wt.shape, out=dW),
        }
        for dname in dirs:
            fn = fns[dname]
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            if args.device_time:
                Fn.TIMER = Fn.LaunchTimer()
                for _ in range(args.iters):
                    fn()
                summ = Fn.TIMER.summary()
                parts = [0.0, 0.0]
                ms = __import__('ctypes').c_float()
                for _, _, _, pairs in Fn.TIMER.rec:
                    for i, (a0, a1) in enumerate(pairs[:2]):
                        Fn.ops.event_elapsed(a0, a1, __import__('ctypes').byref(ms))
                        parts[i] += ms.value * 1e3 / args.iters
                Fn.TIMER = None
                us = sum(v[3] for v in summ.values()) * 1e6 / args.iters
                if parts[1]:
                    print('%-16s %-6s   kernel %7.2f us + reduce %6.2f us' % (name, dname, parts[0], parts[1]))
            else:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / args.iters
            print('%-16s %-6s %9.2f us %8.1f TF/s' % (name, dname, us, flops / us / 1e6), flush=True)


if __name__ == '__main__':
    main()
