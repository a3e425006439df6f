#!/usr/bin/env python
"""In-process A/B of environment knobs on the replayed step graph: one
trainer, settings alternated R times, each setting captured into its own
StepGraph and timed over K replays.  Comparing within one process removes
the per-process spread (~541 vs ~575 img/s between processes
of one build).  Knobs must be read at launch time (the conv planner's are;
module constants such as EEGAN_DAMSM_EARLY are read at import and cannot be
switched this way).  The order of the settings rotates every repetition (the
clock drifts over a run: a fixed order biases the comparison).

    python tools/ab_inproc.py "EEGAN_CONV=mink=32" ["EEGAN_CONV=mink=8" ...] [--reps 3] [--steps 20]
    python tools/ab_inproc.py "py:eegan_hip.functional.FUSE_GP_ADDS=False"   (a module constant)
"""
import argparse
import gc
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'ee-gan_amd'))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def _py_attr(path):
    import importlib
    modname, attr = path.rsplit('.', 1)
    return importlib.import_module(modname), attr


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('settings', nargs='+')
    ap.add_argument('--reps', type=int, default=3)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--config', default='C2')
    args = ap.parse_args()
    import bench
    from eegan_hip.synthetic import make_batch
    from eegan_hip.trainer import StepGraph
    dev = torch.device('cuda', 0)
    torch.autograd.graph.set_warn_on_accumulate_grad_stream_mismatch(False)
    T, B, ncls = bench.build(args.config, dev)
    batch = make_batch(B, dev, seed=3407, class_num=ncls, with_class=True)
    settings = ['base'] + args.settings
    res = {s: [] for s in settings}
    base_env = dict(os.environ)
    py_base = []
    for s in args.settings:
        for kv in s.split():
            if kv.startswith('py:'):
                mod, attr = _py_attr(kv.split('=', 1)[0][3:])
                py_base.append((mod, attr, getattr(mod, attr)))
    for rep in range(args.reps):
        for s in settings[rep % len(settings):] + settings[:rep % len(settings)]:
            os.environ.clear()
            os.environ.update(base_env)
            for mod, attr, v in py_base:
                setattr(mod, attr, v)
            if s != 'base':
                for kv in s.split():
                    k, v = kv.split('=', 1)
                    if k.startswith('py:'):   # py:package.module.ATTR=value (module constants)
                        mod, attr = _py_attr(k[3:])
                        setattr(mod, attr, eval(v))
                    else:
                        os.environ[k] = v
            sg = StepGraph(T, batch, warmup=1)
            sg.replay()
            torch.cuda.synchronize()
            t0 = time.time()
            for _ in range(args.steps):
                sg.replay()
            torch.cuda.synchronize()
            dt = time.time() - t0
            res[s].append(B * args.steps / dt)
            print('rep %d  %-40s %8.1f img/s' % (rep, s, res[s][-1]), flush=True)
            del sg
            gc.collect()
            torch.cuda.empty_cache()
    for s in settings:
        v = res[s]
        print('%-40s mean %8.1f  min %8.1f  max %8.1f  (%+.1f %% vs base)' % (
            s, sum(v) / len(v), min(v), max(v), 100 * (sum(v) / len(v) / (sum(res['base']) / len(res['base'])) - 1)))


if __name__ == '__main__':
    main()
