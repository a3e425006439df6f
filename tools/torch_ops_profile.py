#!/usr/bin/env python
"""Where the step's non-native GPU work comes from: one eager train_step under
torch.profiler (with Python stacks), aggregated per aten op and call stack for
the ops that launch torch's own kernels (adds of gradient accumulation, copies,
fills).  The replayed graph runs the same launches; this only names their
Python call sites.

    python tools/torch_ops_profile.py [--config C2] [--ops aten::add_,aten::copy_]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'ee-gan_amd'))
sys.path.insert(0, REPO)

import torch  # noqa: E402

DEFAULT_OPS = ('aten::add', 'aten::add_', 'aten::copy_', 'aten::cat', 'aten::fill_', 'aten::zero_',
               'aten::mul', 'aten::mul_', 'aten::sum', 'aten::clone', 'aten::div', 'aten::sub')


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='C2')
    ap.add_argument('--ops', default=','.join(DEFAULT_OPS))
    ap.add_argument('--stack', type=int, default=6)
    args = ap.parse_args()
    import bench
    from eegan_hip.synthetic import make_batch
    dev = torch.device('cuda', 0)
    torch.autograd.graph.set_warn_on_accumulate_grad_stream_mismatch(False)
    T, B, ncls = bench.build(args.config, dev)
    batch = make_batch(B, dev, seed=3407, class_num=ncls, with_class=True)
    for _ in range(2):
        T.train_step(batch)
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU]
    with torch.profiler.profile(activities=acts, with_stack=True, record_shapes=True) as prof:
        T.train_step(batch)
        torch.cuda.synchronize()
    ops = set(args.ops.split(','))
    rows = [e for e in prof.key_averages(group_by_stack_n=args.stack) if e.key in ops]
    rows.sort(key=lambda e: -e.count)
    print('%-14s %6s  stack' % ('op', 'calls'))
    for e in rows:
        stack = [s for s in e.stack if 'eegan' in s or 'bench' in s or 'trainer' in s][:args.stack]
        print('%-14s %6d  %s' % (e.key, e.count, ' <- '.join(stack) or '(no python frames)'))
    print()
    shp = [e for e in prof.key_averages(group_by_input_shape=True) if e.key in ops]
    shp.sort(key=lambda e: -e.count)
    for e in shp[:60]:
        print('%-14s %6d  %s' % (e.key, e.count, str(e.input_shapes)[:200]))
    tot = {}
    for e in prof.key_averages():
        if e.key in ops:
            tot[e.key] = e.count
    print('totals', tot)


if __name__ == '__main__':
    main()
