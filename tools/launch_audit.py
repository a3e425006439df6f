"""Which autograd Functions launch which conv / GEMM / BN entry points in each
phase of one training step (diagnostic): the C2 step run eagerly on one
stream with the phase stamps on; the raw entry points of eegan_hip.functional
are wrapped to record (phase, entry point, calling Function).  A phase's
launches are the ones issued between its stamp and the previous one.  Wasted
passes show up as entry points from Functions that should not run in that
phase (round 5: the gradient penalty's second backward walking the forward
graph on zero-filled gradients, tools/gp_trace.py).

    python3 tools/launch_audit.py [--config C2] [--phase SUBSTR]
"""
import argparse
import collections
import inspect
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'ee-gan_amd'))
sys.path.insert(0, REPO)
import torch  # noqa: E402

ENTRY = ('conv_fwd_raw', 'conv_bwd_data_raw', 'conv_bwd_weight_raw', 'chansum_raw', '_gemm', 'act_bwd_raw')


def caller():
    for f in inspect.stack()[2:8]:
        if f.function in ('forward', 'backward'):
            self_cls = f.frame.f_locals.get('ctx')
            cls = type(self_cls).__name__ if self_cls is not None else '?'
            return '%s.%s:%d' % (cls.replace('Backward', ''), f.function, f.lineno)
    f = inspect.stack()[2]
    return '%s:%d' % (f.function, f.lineno)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='C2')
    ap.add_argument('--phase', default='')
    args = ap.parse_args()
    import bench
    from eegan_hip import functional as Fn
    from eegan_hip.synthetic import make_batch
    dev = torch.device('cuda', 0)
    T, B, ncls = bench.build(args.config, dev)
    T.use_streams = False
    batch = make_batch(B, dev, class_num=ncls, with_class=True)
    T.train_step(batch)
    torch.cuda.synchronize()
    pending = []
    table = collections.OrderedDict()
    active = [False]
    for name in ENTRY:
        orig = getattr(Fn, name, None)
        if orig is None:
            continue

        def w(*a, _o=orig, _n=name, **k):
            if active[0]:
                pending.append((_n, caller()))
            return _o(*a, **k)
        setattr(Fn, name, w)
    ostamp = Fn.stamp

    def stamp(name):
        if active[0]:
            c = table.setdefault(name, collections.Counter())
            for e in pending:
                c[e] += 1
            pending.clear()
        return ostamp(name)
    Fn.stamp = stamp
    Fn.STAMP_BUF = torch.zeros(4096, dtype=torch.int64, device=dev)
    Fn.STAMPS = []
    active[0] = True
    T.train_step(batch)
    active[0] = False
    Fn.STAMPS = None
    torch.cuda.synchronize()
    for ph, c in table.items():
        if args.phase and args.phase not in ph:
            continue
        print('== %s: %d launches' % (ph, sum(c.values())))
        for (n, who), k in sorted(c.items(), key=lambda kv: (kv[0][0], -kv[1])):
            print('  %3d  %-20s %s' % (k, n, who))


if __name__ == '__main__':
    main()
