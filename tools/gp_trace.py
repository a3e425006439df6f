"""Which autograd Functions launch data / weight gradients during the gradient
penalty's second backward (diagnostic): one Dis256 GP at C2 size, the conv
entry points wrapped to record their calling Function.

    python3 tools/gp_trace.py
"""
import collections
import inspect
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'ee-gan_amd'))
sys.path.insert(0, REPO)
import torch  # noqa: E402

ACTIVE = [False]


def main():
    import bench
    from eegan_hip import functional as Fn
    from eegan_hip.synthetic import make_batch
    dev = torch.device('cuda', 0)
    T, B, ncls = bench.build('C2', dev)
    batch = make_batch(B, dev, seed=3, class_num=ncls, with_class=True)
    sent = torch.randn(B, 256, device=dev)
    netD = T.netsD[2]
    counts = collections.Counter()
    wrapped = {}
    for name in ('conv_bwd_weight_raw', 'conv_bwd_data_raw', 'conv_fwd_raw'):
        orig = getattr(Fn, name)
        wrapped[name] = orig

        def w(*a, _o=orig, _n=name, **k):
            if ACTIVE[0]:
                st = inspect.stack()
                who = [f.function + ':' + os.path.basename(f.filename) + ':' + str(f.lineno) for f in st[1:4]]
                counts[(_n, ' <- '.join(who))] += 1
            return _o(*a, **k)
        setattr(Fn, name, w)
    gp = T.MA_gradient_penalty(batch['imgs'][2], sent, netD, True)
    ACTIVE[0] = True
    T.optimizerDs[2].zero_grad()
    gp.backward(inputs=T.optimizerDs[2].params)
    torch.cuda.synchronize()
    for (n, who), c in sorted(counts.items(), key=lambda kv: -kv[1]):
        print('%3d  %-20s %s' % (c, n, who))


if __name__ == '__main__':
    main()
