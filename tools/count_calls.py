#!/usr/bin/env python
"""Which C-ABI entry points (and which torch kernels) one eager bench step
issues, counted by (entry point, calling Function): the launch budget of the
step, to direct fusion work.

    python tools/count_calls.py [--config C2]
"""
import argparse
import collections
import os
import sys
import traceback

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'ee-gan_amd'))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='C2')
    args = ap.parse_args()
    import bench
    from eegan_hip import _lib
    from eegan_hip.synthetic import make_batch
    dev = torch.device('cuda', 0)
    T, B, ncls = bench.build(args.config, dev)
    batch = make_batch(B, dev, class_num=ncls)
    T.train_step(batch)
    torch.cuda.synchronize()
    cnt = collections.Counter()
    orig = {}

    def wrap(name, fn):
        def call(*a):
            st = traceback.extract_stack(limit=6)[:-1]
            where = '/'.join('%s:%s' % (os.path.basename(f.filename), f.name) for f in st[-3:])
            cnt[(name, where)] += 1
            return fn(*a)
        return call

    for name in list(vars(_lib.ops)):
        if name.endswith('workspace') or name in ('last_error', 'abi_version'):
            continue
        orig[name] = getattr(_lib.ops, name)
        setattr(_lib.ops, name, wrap(name, orig[name]))
    from torch.profiler import profile, ProfilerActivity
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        T.train_step(batch)
        torch.cuda.synchronize()
    for name, fn in orig.items():
        setattr(_lib.ops, name, fn)
    tot = sum(cnt.values())
    print('C-ABI calls per step: %d' % tot)
    for (name, where), n in cnt.most_common(70):
        print('%5d  %-24s %s' % (n, name, where))
    kc = collections.Counter()
    for ev in prof.events():
        if ev.device_type == torch.autograd.DeviceType.CUDA:
            kc[ev.name[:90]] += 1
    print('\nGPU kernels per step: %d' % sum(kc.values()))
    for k, n in kc.most_common(45):
        print('%5d  %s' % (n, k))


if __name__ == '__main__':
    main()
