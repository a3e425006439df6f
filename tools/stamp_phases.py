#!/usr/bin/env python
"""Device-side phase timing of the REPLAYED step graph (bench.py's execution
mode): one-thread stamp kernels (eegan_stamp, the 100 MHz device clock) at the
Trainer's phase boundaries, captured into the graph with everything else, read
back after a replay.  Prints, per stream lane, each phase's duration (time
from the lane's previous stamp) and its start / end relative to the step's
start, so the critical path through the concurrent D lanes is visible.

    python tools/stamp_phases.py [--config C2] [--replays 5]
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
    ap.add_argument('--replays', type=int, default=5)
    args = ap.parse_args()
    import bench
    from eegan_hip import functional as Fn
    from eegan_hip.synthetic import make_batch
    from eegan_hip.trainer import StepGraph
    dev = torch.device('cuda', 0)
    T, B, ncls = bench.build(args.config, dev)
    batch = make_batch(B, dev, class_num=ncls, with_class=True)
    Fn.STAMP_BUF = torch.zeros(4096, dtype=torch.int64, device=dev)
    Fn.STAMPS = None
    torch.autograd.graph.set_warn_on_accumulate_grad_stream_mismatch(False)
    # stamps only inside the captured step (warm-up steps run unstamped)
    orig = T.train_step

    def stamped(*a, **k):
        Fn.STAMPS = [] if capturing[0] else None
        try:
            return orig(*a, **k)
        finally:
            if capturing[0]:
                names[:] = Fn.STAMPS
            Fn.STAMPS = None
    capturing = [False]
    names = []
    T.train_step = stamped
    _enter = torch.cuda.graph.__enter__

    def enter(self):
        capturing[0] = True
        return _enter(self)
    torch.cuda.graph.__enter__ = enter
    sg = StepGraph(T, batch, warmup=1)
    capturing[0] = False
    acc = collections.defaultdict(float)
    spans = collections.defaultdict(lambda: [0.0, 0.0])
    total = 0.0
    for r in range(args.replays + 1):
        sg.replay()
        torch.cuda.synchronize()
        if r == 0:
            continue
        ts = Fn.STAMP_BUF[:len(names)].cpu().tolist()
        t0 = ts[0]
        last = {}
        for (name, st), t in zip(names, ts):
            if name == 'start':
                last[st] = t
                continue
            prev = last.get(st, t0)
            acc[name] += (t - prev) / 100.0 / args.replays      # 100 MHz -> us
            spans[name][0] += (prev - t0) / 100.0 / args.replays
            spans[name][1] += (t - t0) / 100.0 / args.replays
            last[st] = t
        total += (ts[[n for n, _ in names].index('end')] - t0) / 100.0 / args.replays
    lanes = {}
    for name, st in names:
        lanes.setdefault(st, len(lanes))
    print('%-28s %4s %10s %10s %10s' % ('phase (ends at stamp)', 'lane', 'dur us', 'from us', 'to us'))
    seen = set()
    for name, st in names:
        if name == 'start' or name in seen:
            continue
        seen.add(name)
        print('%-28s %4d %10.1f %10.1f %10.1f' % (name, lanes[st], acc[name], spans[name][0], spans[name][1]))
    print('step (start -> end stamp): %.1f us' % total)


if __name__ == '__main__':
    main()
