"""Diagnose eager-vs-graph step differences (T8 config): eager twice, graph once."""
import os
import sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'ee-gan_amd'))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'tests'))
import torch  # noqa: E402


def run(mode, steps):
    import bench
    from eegan_hip.trainer import StepGraph
    from eegan_hip.synthetic import make_batch
    from oracle.seeding import seeded_tensor
    dev = torch.device('cuda', 0)
    T, B, ncls = bench.build('T8', dev, sim_coe=0.0)
    batch = make_batch(B, dev, seed=11, class_num=ncls, with_class=True)
    noise = seeded_tensor('graph:noise', (B, 100), 1).to(dev)
    if mode == 'eager':
        for _ in range(steps):
            T.train_step(batch, noise=noise)
    else:
        sg = StepGraph(T, batch, warmup=1, noise=noise)
        for _ in range(steps - 1):
            sg.replay()
    torch.cuda.synchronize()
    return [o.flat.clone() for o in [T.optimizerG] + list(T.optimizerDs)]


for steps in (1, 2, 3):
    a = run('eager', steps)
    b = run('eager', steps)
    c = run('graph', steps) if steps > 1 else None
    print('steps', steps, 'eager-eager', ['%.2e' % float((x - y).abs().max()) for x, y in zip(a, b)])
    if c is not None:
        print('steps', steps, 'graph-eager', ['%.2e' % float((x - y).abs().max()) for x, y in zip(a, c)])
