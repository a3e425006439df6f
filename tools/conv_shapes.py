#!/usr/bin/env python
"""Per-shape conv time of one eager C2 step (single stream, HIP events per
dispatch, functional.LaunchTimer(detail=True)): which conv shapes and
directions the step's conv time goes to, so kernel work can be aimed.

    python tools/conv_shapes.py [--config C2] [--steps 2] [--top 60]
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
    ap.add_argument('--config', default='C2')
    ap.add_argument('--steps', type=int, default=2)
    ap.add_argument('--top', type=int, default=60)
    args = ap.parse_args()
    import bench
    from eegan_hip import functional as Fn
    from eegan_hip.synthetic import make_batch
    dev = torch.device('cuda', 0)
    T, B, ncls = bench.build(args.config, dev)
    batch = make_batch(B, dev, seed=3407, class_num=ncls, with_class=True)
    T.use_streams = False
    for _ in range(2):
        T.train_step(batch)
    torch.cuda.synchronize()
    timer = Fn.LaunchTimer(detail=True)
    Fn.TIMER = timer
    for _ in range(args.steps):
        T.train_step(batch)
    Fn.TIMER = None
    summ = timer.summary()
    rows = sorted(((v[3] / args.steps, k, v) for k, v in summ.items()), key=lambda r: -r[0])
    tot = sum(r[0] for r in rows if isinstance(r[1], tuple) and str(r[1][0]).startswith('conv'))
    print('conv total %.3f ms/step' % (tot * 1e3))
    for t, k, v in rows[:args.top]:
        kind, key = k if isinstance(k, tuple) else (k, '')
        n = v[0] // args.steps
        print('%7.3f ms %4d x %7.2f us %7.1f TF  %-14s %s' % (t * 1e3, n, t / max(n, 1) * 1e6,
                                                           v[1] / max(v[3], 1e-12) / 1e12, kind, key))


if __name__ == '__main__':
    main()
