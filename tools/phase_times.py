#!/usr/bin/env python
"""Per-phase device time of one eager bench step on ONE stream (text encode,
ATTR + G forward, each D's d_update, g_update's D passes, the DAMSM image
encoder + losses, G backward + Adam): where the step's time goes.

    python tools/phase_times.py [--config C2] [--steps 3]
"""
import argparse
import collections
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'ee-gan_amd'))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='C2')
    ap.add_argument('--steps', type=int, default=3)
    args = ap.parse_args()
    import bench
    from eegan_hip.synthetic import make_batch
    from eegan_hip import trainer as TR
    dev = torch.device('cuda', 0)
    T, B, ncls = bench.build(args.config, dev)
    T.use_streams = False
    batch = make_batch(B, dev, class_num=ncls)
    marks = []

    def mark(name):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        marks.append((name, e))

    # mark the boundaries of the Trainer's phases (intervals are labelled by their end mark)
    def wrap(n, label):
        f = getattr(TR.Trainer, n)

        def g(self, *a, **k):
            mark('before ' + (label(a) if callable(label) else label))
            r = f(self, *a, **k)
            mark(label(a) if callable(label) else label)
            return r
        setattr(TR.Trainer, n, g)

    wrap('encode_text', 'text encode')
    wrap('d_update', 'd_update (3 D)')
    wrap('_d_update_one', lambda a: 'D%d update' % a[0])
    wrap('DAMSM_loss', 'DAMSM (Inception + losses)')
    og = T.optimizerG.step

    def gstep(*a, **k):
        mark('g backward')
        r = og(*a, **k)
        mark('g adam')
        return r
    T.optimizerG.step = gstep
    acc = collections.OrderedDict()
    for it in range(args.steps + 1):
        marks.clear()
        torch.cuda.synchronize()
        mark('start')
        T.train_step(batch)
        mark('end')
        torch.cuda.synchronize()
        if it == 0:
            continue
        for (n0, e0), (n1, e1) in zip(marks[:-1], marks[1:]):
            acc[n1] = acc.get(n1, 0.0) + e0.elapsed_time(e1) / args.steps
    tot = sum(acc.values())
    for n, v in acc.items():
        print('%-22s %8.3f ms  %5.1f%%' % (n, v, 100 * v / tot))
    print('%-22s %8.3f ms' % ('total (1 stream)', tot))


if __name__ == '__main__':
    main()
