#!/usr/bin/env python
"""Which torch-native (aten) ops still run inside the bench step, and from where:
one eager step under torch.profiler, aten ops grouped by (name, python caller).

    python tools/torch_ops_profile.py [--config C2]
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
    args = ap.parse_args()
    import bench
    from eegan_hip.synthetic import make_batch
    dev = torch.device('cuda', 0)
    T, B, ncls = bench.build(args.config, dev)
    batch = make_batch(B, dev, class_num=max(ncls, 1))
    T.train_step(batch)
    torch.cuda.synchronize()
    from torch.profiler import profile, ProfilerActivity
    with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=True) as prof:
        T.train_step(batch)
        torch.cuda.synchronize()
    cnt = collections.Counter()
    for ev in prof.events():
        if not ev.name.startswith('aten::') or ev.name in ('aten::empty', 'aten::empty_strided', 'aten::as_strided',
                                                          'aten::view', 'aten::permute', 'aten::slice',
                                                          'aten::select', 'aten::detach', 'aten::alias',
                                                          'aten::t', 'aten::transpose', 'aten::expand',
                                                          'aten::unsqueeze', 'aten::squeeze', 'aten::reshape',
                                                          'aten::_reshape_alias', 'aten::lift_fresh',
                                                          'aten::resolve_conj', 'aten::resolve_neg',
                                                          'aten::result_type', 'aten::to', 'aten::is_nonzero',
                                                          'aten::item', 'aten::_local_scalar_dense', 'detach',
                                                          'aten::empty_like', 'aten::contiguous',
                                                          'aten::_unsafe_view', 'aten::unbind', 'aten::split',
                                                          'aten::narrow', 'aten::chunk', 'aten::numpy_T',
                                                          'aten::set_', 'aten::new_empty_strided',
                                                          'aten::new_empty', 'aten::zeros_like_', 'aten::flatten'):
            continue
        stack = [f for f in (ev.stack or []) if 'site-packages' not in f and 'torch/' not in f]
        where = ' < '.join(stack[:3]) if stack else '?'
        shapes = str(ev.input_shapes)[:60] if ev.input_shapes else ''
        cnt[(ev.name, where, shapes)] += 1
    for (name, where, shapes), n in cnt.most_common(60):
        print('%4d  %-28s %-60s %s' % (n, name, shapes, where))


if __name__ == '__main__':
    main()
