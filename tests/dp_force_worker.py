"""One rank (torchrun --nproc-per-node 1) of the data-parallel trainer step
with EEGAN_FORCE_DIST=1: every collective of the N > 1 step -- SyncBN
statistics, DAMSM gathers, the gradient buckets -- is issued over RCCL
(one-rank communicators of eegan_hip.rccl, one per stream lane) and captured
in the step graph.  mode 'eager': 3 eager steps; 'graph': 1 eager + capture +
2 replays; trainer.COMM_LANES from DP_COMM_LANES.  Writes every optimizer's
parameters and Adam moments to OUT/force_<tag>.pt (tests/test_gpu_dist.py)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in (REPO, os.path.join(REPO, 'ee-gan_amd'), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402


def main(out, tag, mode):
    assert os.environ.get('EEGAN_FORCE_DIST') == '1'
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    import bench
    from eegan_hip import trainer as TR
    from eegan_hip import dist as D
    from eegan_hip.synthetic import make_batch
    from oracle.seeding import seeded_tensor
    TR.COMM_LANES = os.environ.get('DP_COMM_LANES', '1') == '1'
    rank, world = D.init_from_env()
    assert world == 1 and D.collective() and len(D.COMMS) == D.N_LANES, (world, len(D.COMMS))
    T, B, ncls = bench.build('T8', dev, sim_coe=0.05)
    batch = make_batch(B, dev, seed=11, class_num=ncls, with_class=True)
    noise = seeded_tensor('graph:noise', (B, 100), 1).to(dev)
    if mode == 'eager':
        for _ in range(3):
            T.train_step(batch, noise=noise)
    else:
        sg = TR.StepGraph(T, batch, warmup=1, noise=noise)
        sg.replay()
        sg.replay()
    torch.cuda.synchronize()
    opts = [T.optimizerG] + list(T.optimizerDs)
    torch.save({'state': torch.cat([o.flat for o in opts] + [o.v for o in opts]).cpu(),
                'comm_lanes': [o.comm_stream is not None for o in opts]},
               os.path.join(out, 'force_%s.pt' % tag))


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2], sys.argv[3])
