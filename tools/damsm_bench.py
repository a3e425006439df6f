#!/usr/bin/env python
"""Microbenchmark of the DAMSM words similarity (csrc/damsm.hip) at the bench
shapes: C2 (16 images x 16 captions, one GPU) and the C5 shard (32 local
images x 256 global captions).  Times forward and forward+backward (incl. the
dregions GEMM) with torch.cuda events around R replays of a captured graph of
the call (device time, as in the graph-replayed bench step; --eager times
back-to-back eager calls, host launch overhead included).

    python tools/damsm_bench.py [--reps 20] [--out profiles/r02_damsm_bench.json]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'ee-gan_amd'))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def bench(n_img, n_txt, T, reps, dev, eager=False):
    from eegan_hip import functional as Fn
    from eegan_hip.tensor import empty_nhwc
    torch.manual_seed(0)
    reg = empty_nhwc(n_img, 256, 17, 17, dev, dtype=torch.float32)
    reg.copy_(torch.randn(n_img, 256, 17, 17, device=dev) * 0.3)
    words = torch.randn(n_txt, 256, T, device=dev).tanh()
    lens = torch.randint(5, T + 1, (n_txt,), device=dev)
    dsim = torch.randn(n_img, n_txt, device=dev)
    regg = reg.detach().requires_grad_()

    def fwd():
        return Fn.WordsSimFn.apply(reg, words, lens, False, 0)[0]

    def fwdbwd():
        sim, _ = Fn.WordsSimFn.apply(regg, words, lens, False, 0)
        sim.backward(dsim)

    out = {}
    for name, fn in (('fwd', fwd), ('fwd_bwd', fwdbwd)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        if not eager:
            g = torch.cuda.CUDAGraph()
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                regg.grad = None
                fn()
                torch.cuda.synchronize()
                regg.grad = None
                with torch.cuda.graph(g):
                    fn()
            torch.cuda.synchronize()
            fn = g.replay
            fn()
            torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out[name + '_us'] = round(e0.elapsed_time(e1) * 1e3 / reps, 2)
    pairs = n_img * n_txt
    # algorithmic MFMA work per pair at the padded shapes the kernel runs:
    # S 3 x 2*304*256*32 (split bf16), C 2*320*256*32; backward adds dA2 2*304*256*32 and
    # the dregions GEMM 2*304*256*64 (per caption); the backward's recompute of
    # the forward is not counted
    f_fwd = pairs * (3 * 2 * 304 * 256 * 32 + 2 * 320 * 256 * 32)
    f_bwd = pairs * (2 * 304 * 256 * 32 + 2 * 304 * 256 * 64)
    out.update(n_img=n_img, n_txt=n_txt, T=T, pairs=pairs,
               fwd_TFLOPs=round(f_fwd / out['fwd_us'] / 1e6, 1),
               fwd_bwd_TFLOPs=round((f_fwd + f_bwd) / out['fwd_bwd_us'] / 1e6, 1))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=20)
    ap.add_argument('--out', default=None)
    ap.add_argument('--eager', action='store_true')
    args = ap.parse_args()
    dev = torch.device('cuda:0')
    res = {'C2 (16 x 16, T 18)': bench(16, 16, 18, args.reps, dev, args.eager),
           'C5 shard (32 local x 256 global, T 18)': bench(32, 256, 18, max(3, args.reps // 4), dev, args.eager),
           'timing': 'eager calls' if args.eager else 'graph replay (device time)'}
    s = json.dumps(res, indent=1)
    print(s)
    if args.out:
        with open(args.out, 'w') as f:
            f.write(s + '\n')


if __name__ == '__main__':
    main()
