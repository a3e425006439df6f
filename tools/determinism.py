#!/usr/bin/env python
"""Run-to-run determinism of the step: build the bench workload from fixed
seeds R times in one process, run K eager steps (or 1 eager + K-1 replays with
--graph), and compare every optimizer's parameters and Adam moments with the
first run's -- bit for bit.  Prints the max |diff| per optimizer per run.

    python tools/determinism.py [--config C2] [--reps 4] [--steps 2] [--graph]
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
    ap.add_argument('--reps', type=int, default=4)
    ap.add_argument('--steps', type=int, default=2)
    ap.add_argument('--graph', action='store_true')
    ap.add_argument('--nostreams', action='store_true')
    args = ap.parse_args()
    import bench
    from eegan_hip.trainer import StepGraph
    from eegan_hip.synthetic import make_batch
    from oracle.seeding import seeded_tensor
    dev = torch.device('cuda', 0)
    first = None
    names = ['G', 'D0', 'D1', 'D2']
    for r in range(args.reps):
        T, B, ncls = bench.build(args.config, dev, sim_coe=0.05)
        if args.nostreams:
            T.use_streams = False
        batch = make_batch(B, dev, seed=11, class_num=ncls, with_class=True)
        noise = seeded_tensor('graph:noise', (B, 100), 1).to(dev)
        if args.graph:
            sg = StepGraph(T, batch, warmup=1, noise=noise)
            for _ in range(args.steps - 1):
                sg.replay()
        else:
            for _ in range(args.steps):
                T.train_step(batch, noise=noise)
        torch.cuda.synchronize()
        opts = [T.optimizerG] + list(T.optimizerDs)
        st = [(o.flat.clone(), o.v.clone()) for o in opts]
        gnames = {}
        for mod, tag in ((T.netG, 'G'), (T.attr_enhance, 'A')):
            for n_, p_ in getattr(mod, 'module', mod).named_parameters():
                gnames[id(p_)] = tag + '.' + n_
        gparams = [(gnames.get(id(p_), '?'), p_.detach().float().clone()) for p_ in T.optimizerG.params]
        if first is None:
            first = st
            first_g = gparams
        else:
            d = ['%s %.3e/%.3e' % (n, float((a[0] - b[0]).abs().max()), float((a[1] - b[1]).abs().max()))
                 for n, a, b in zip(names, st, first)]
            print('determinism run %d vs run 0 (param/moment max|diff|): %s' % (r, '  '.join(d)), flush=True)
            diffs = sorted(((float((a - b).abs().max()), n) for (n, a), (_, b) in zip(gparams, first_g)), reverse=True)
            bad = [(n, e) for e, n in diffs if e > 0]
            if bad:
                print('   G params differing: %d of %d; top: %s' % (len(bad), len(diffs),
                      ', '.join('%s %.1e' % (n, e) for n, e in bad[:12])), flush=True)
        del T
        if args.graph:
            del sg


if __name__ == '__main__':
    main()
