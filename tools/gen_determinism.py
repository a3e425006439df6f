#!/usr/bin/env python
"""Run-to-run determinism of the generator alone at the C2 width (W=32, B=16):
forward_branched (stage 2-3 branches on a second stream) + backward from
fixed seeded weights and inputs, repeated; every parameter gradient compared
bit for bit with the first repetition.  --single: one stream.

    python tools/gen_determinism.py [--reps 20] [--single]
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
    ap.add_argument('--reps', type=int, default=20)
    ap.add_argument('--single', action='store_true')
    ap.add_argument('--load', action='store_true', help='a busy side stream beside the backward')
    args = ap.parse_args()
    import models
    from oracle.seeding import seeded_state, state_spec, seeded_tensor
    dev = torch.device('cuda', 0)
    G = models.Gen(32, 100)
    G.load_state_dict(seeded_state(state_spec(G.state_dict()), 21))
    G = G.to(dev)
    z = seeded_tensor('g:z', (16, 100), 1).to(dev)
    s = seeded_tensor('g:s', (16, 256), 1).to(dev)
    a = seeded_tensor('g:a', (16, 256), 1).to(dev)
    rs = [seeded_tensor('g:r%d' % k, (16, 3, 64 << k, 64 << k), 2).to(dev) for k in range(3)]
    G.side_stream = None if args.single else torch.cuda.Stream()
    ref, bad = None, 0
    bg = torch.cuda.Stream()
    big = torch.randn(32 << 20, device=dev)
    for r in range(args.reps):
        G.zero_grad(set_to_none=True)
        if args.load:   # a stream hammering memory beside the whole pass
            with torch.cuda.stream(bg):
                for _ in range(60):
                    big.mul_(1.0000001)
        imgs = G(z, s, a)
        loss = sum((im.float() * rk).sum() for im, rk in zip(imgs, rs))
        loss.backward()
        torch.cuda.synchronize()
        gr = {n: p.grad.clone() for n, p in G.named_parameters() if p.grad is not None}
        im = [i.float().clone() for i in imgs]
        if ref is None:
            ref = (gr, im)
            continue
        dimg = [float((x - y).abs().max()) for x, y in zip(im, ref[1])]
        diff = sorted(((float((gr[n] - ref[0][n]).abs().max()), n) for n in gr), reverse=True)
        nb = sum(1 for e, _ in diff if e > 0)
        if nb or any(dimg):
            if bad == 0:
                same = sorted({n.rsplit('.', 1)[0].split('.affine')[0] for e, n in diff if e == 0})
                dif = sorted({n.rsplit('.', 1)[0].split('.affine')[0] for e, n in diff if e > 0})
                print('gen determinism: identical modules %s' % same)
                print('gen determinism: differing modules %s' % dif)
                print('gen determinism: blocks.5/6 params: %s' % ['%s %s' % (n, 'DIFF' if e > 0 else 'same')
                                                             for e, n in diff if n.startswith(('blocks.5', 'blocks.4.c2', 'blocks.4.gamma'))])
            bad += 1
            print('gen determinism rep %d: images max|d| %s; %d params differ, top %s' % (
                r, ['%.1e' % d for d in dimg], nb, ', '.join('%s %.1e' % (n, e) for e, n in diff[:6])), flush=True)
    print('gen determinism: %d of %d repetitions differ (%s)' % (bad, args.reps - 1,
                                                                 'one stream' if args.single else 'branched'))


if __name__ == '__main__':
    main()
