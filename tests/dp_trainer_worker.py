"""Two eager steps of the eegan_hip.trainer path (FlatAdam, the bench's
optimizer) on one rank of a torchrun group; writes every parameter after the
steps and how many gradient buckets each optimizer reduced DURING a backward
(FlatAdam's overlapped all-reduce) to OUT/rankR_<tag>.pt.  The first step's
windows learn the write plans, the second overlaps.  tests/test_gpu_dist.py
runs it with EEGAN_GRAD_OVERLAP=1 and =0, and with the generator's second
stream (trainer.GEN_SIDE) and the communication lanes (trainer.COMM_LANES)
off (DP_GEN_SIDE=0, DP_COMM_LANES=0), two ranks sharing one GPU over gloo, and
requires bit-identical parameters."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in (REPO, os.path.join(REPO, 'ee-gan_amd'), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402


def main(out, tag):
    os.environ.setdefault('EEGAN_DIST_BACKEND', 'gloo')
    os.environ.setdefault('EEGAN_SHARE_GPU', '1')
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    import bench
    from eegan_hip import trainer as TR
    from eegan_hip import dist as D
    TR.GEN_SIDE = os.environ.get('DP_GEN_SIDE', '1') == '1'
    TR.COMM_LANES = os.environ.get('DP_COMM_LANES', '1') == '1'
    from eegan_hip import optim as O
    from eegan_hip.synthetic import make_batch
    rank, world = D.init_from_env()
    early = {}
    orig = O.FlatAdam._reduce_bucket

    def counted(self, b):   # reductions issued from inside a backward (a window still open with its plan)
        w = self._win
        if w is not None and w['cands'] and not getattr(self, '_in_step', False):
            early[id(self)] = early.get(id(self), 0) + 1
        return orig(self, b)
    O.FlatAdam._reduce_bucket = counted
    ostep = O.FlatAdam._allreduce

    def in_step(self):
        self._in_step = True
        try:
            return ostep(self)
        finally:
            self._in_step = False
    O.FlatAdam._allreduce = in_step
    torch.manual_seed(1234)
    T, B, ncls = bench.build('T8', dev)
    for o in [T.optimizerG] + list(T.optimizerDs):
        o.set_bucket_bytes(16384)   # many small buckets at this test size
    batch = make_batch(B, dev, seed=11 + rank, class_num=ncls, with_class=True, id_offset=rank * B)
    noise = torch.randn(B, 100, device=dev, generator=torch.Generator(device=dev).manual_seed(5 + rank))
    for _ in range(3):   # a write plan steers early reductions from its key's third window on
        T.train_step(batch, noise=noise)
    torch.cuda.synchronize()
    opts = [T.optimizerG] + list(T.optimizerDs)
    if os.environ.get('DP_DEBUG') and rank == 0:
        for o in opts:
            print('DBG opt params %d buckets %d late %d plans %s' % (
                len(o.params), len(o.buckets), len(o._late),
                [(k, sum(e), sum(1 for n in need if n == 0), sorted(set(need))) for k, pl in o._plans.items()
                 for need, e, _ in pl]),
                flush=True)
    torch.save({'params': [o.flat.cpu() for o in opts], 'early': [early.get(id(o), 0) for o in opts],
                'buckets': [len(o.buckets) for o in opts],
                'comm_lanes': [o.comm_stream is not None for o in opts]}, os.path.join(out, 'rank%d_%s.pt' % (rank, tag)))


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
