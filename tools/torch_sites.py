#!/usr/bin/env python
"""Where do the step's torch-issued kernels come from?  Runs eager train steps
of the bench workload under a TorchFunctionMode that records every torch call
made from this package (function name, innermost ee-gan_amd frame) and prints
the counts per step, largest first.  Autograd's own gradient accumulation
(the `add` kernels of multi-consumer tensors) happens in C++ and is not seen
here; `--grad-acc` counts those by hooking every saved activation... (not
needed: their number is the trace's CUDAFunctor_add count minus these).

    python tools/torch_sites.py [--config C2] [--steps 2]
"""
import argparse
import collections
import os
import sys
import traceback

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, 'ee-gan_amd')
sys.path.insert(0, PKG)
sys.path.insert(0, REPO)

import torch  # noqa: E402
from torch.overrides import TorchFunctionMode  # noqa: E402

SKIP = {'__get__', 'data_ptr', 'dim', 'size', 'stride', 'is_contiguous', 'numel', '__len__', 'element_size',
        'storage_offset', 'is_floating_point', 'requires_grad_', 'detach', 'view', 'reshape', 'unflatten',
        'flatten', 'unsqueeze', 'squeeze', 'expand', 'narrow', '__getitem__', 'view_as', 'split', 'chunk',
        'permute', 'transpose', 't', 'as_strided', 'retain_grad', 'register_hook', 'untyped_storage',
        '__format__', '__repr__', 'tolist', 'dtype', 'device', 'shape', 'is_cuda', 'grad', 'requires_grad',
        '_version', 'is_leaf', 'grad_fn', 'data', 'T', 'layout', 'ndim', 'names', '__hash__', '__eq__'}


class Sites(TorchFunctionMode):
    def __init__(self):
        super().__init__()
        self.count = collections.Counter()

    def __torch_function__(self, func, types, args=(), kwargs=None):
        name = getattr(func, '__name__', str(func))
        if name not in SKIP:
            site = '?'
            for fr in reversed(traceback.extract_stack(limit=12)[:-1]):
                if fr.filename.startswith(PKG) or fr.filename.startswith(os.path.join(REPO, 'bench')):
                    site = '%s:%d' % (os.path.relpath(fr.filename, REPO), fr.lineno)
                    break
            self.count[(name, site)] += 1
        return func(*args, **(kwargs or {}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='C2')
    ap.add_argument('--steps', type=int, default=2)
    args = ap.parse_args()
    import bench
    from eegan_hip.synthetic import make_batch
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    T, B, ncls = bench.build(args.config, dev)
    batch = make_batch(B, dev, seed=3407, class_num=ncls, with_class=True)
    torch.autograd.graph.set_warn_on_accumulate_grad_stream_mismatch(False)
    T.train_step(batch)          # warm-up (plans, packs, tickets)
    torch.cuda.synchronize()
    m = Sites()
    with m:
        for _ in range(args.steps):
            T.train_step(batch)
    torch.cuda.synchronize()
    tot = sum(m.count.values()) / args.steps
    print('torch calls per step from the package: %.0f' % tot)
    for (name, site), c in m.count.most_common(60):
        print('%7.1f  %-24s %s' % (c / args.steps, name, site))


if __name__ == '__main__':
    main()
