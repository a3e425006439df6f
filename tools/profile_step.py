#!/usr/bin/env python
"""Per-shape conv timing of the bench workload (HIP events around every conv
launch of N steps): which (direction, shape) pairs dominate the step.

    python tools/profile_step.py [--config C2] [--steps 2] [--out gpurun_out/shapes.json]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'ee-gan_amd'))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='C2')
    ap.add_argument('--steps', type=int, default=2)
    ap.add_argument('--out', default='gpurun_out/shapes.json')
    args = ap.parse_args()
    import bench
    from eegan_hip import functional as Fn
    from eegan_hip.synthetic import make_batch
    dev = torch.device('cuda', 0)
    T, B, ncls = bench.build(args.config, dev)
    batch = make_batch(B, dev, class_num=max(ncls, 1))
    T.train_step(batch)
    torch.cuda.synchronize()
    Fn.TIMER = Fn.LaunchTimer(detail=True)
    for _ in range(args.steps):
        T.train_step(batch)
    torch.cuda.synchronize()
    s = Fn.TIMER.summary()
    Fn.TIMER = None
    rows = []
    for (kind, key), (n, fl, nb, t) in s.items():
        rows.append({'kind': kind, 'shape': key, 'calls_per_step': n / args.steps, 'ms_per_step': t / args.steps * 1e3,
                     'TFLOPs': fl / t / 1e12, 'GBs': nb / t / 1e9})
    rows.sort(key=lambda r: -r['ms_per_step'])
    tot = sum(r['ms_per_step'] for r in rows)
    os.makedirs(os.path.dirname(args.out) or '.', exist_ok=True)
    with open(args.out, 'w') as f:
        json.dump({'total_conv_ms_per_step': tot, 'rows': rows}, f, indent=1)
    print('total conv ms/step %.2f' % tot)
    for r in rows[:40]:
        print('%-15s %-45s x%-5.1f %8.3f ms %7.1f TF %7.1f GB/s' % (r['kind'], r['shape'], r['calls_per_step'],
                                                                 r['ms_per_step'], r['TFLOPs'], r['GBs']))


if __name__ == '__main__':
    main()
