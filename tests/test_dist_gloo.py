"""Data-parallel plumbing on CPU: world_size-2 process groups over gloo
(127.0.0.1).  Covers what the N>1 bench path adds on top of the 1-GPU step:
the differentiable all-gather behind global-batch DAMSM, gradient averaging
(FlatAdam's bucketed all-reduce and GradReducer), and the cross-rank SyncBN
statistics combine (fp64 sums all-reduced, then the reference's multi-device
formula, sync_batchnorm/batchnorm.py:113-125) against the oracle."""
import os
import shutil
import sys
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from _util import REPO

WORLD = 2


def _run(fn, *args, world=WORLD):
    # a file:// store under a fresh directory: no TCP port to pick and lose
    # to another bind between the pick and the store's own bind
    d = tempfile.mkdtemp(prefix='eegan_gloo_')
    try:
        mp.spawn(_entry, args=(fn, 'file://' + os.path.join(d, 'store'), args, world), nprocs=world, join=True)
    finally:
        shutil.rmtree(d, ignore_errors=True)


def _entry(rank, fn, init_method, args, world):
    sys.path.insert(0, os.path.join(REPO, 'ee-gan_amd'))
    sys.path.insert(0, REPO)
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(1)
    dist.init_process_group('gloo', init_method=init_method, rank=rank, world_size=world)
    try:
        fn(rank, *args)
    finally:
        dist.destroy_process_group()


# ----------------------------------------------------------------- cases ---
def _case_all_gather(rank):
    from eegan_hip import dist as D
    torch.manual_seed(100 + rank)
    x = torch.randn(3, 5, requires_grad=True)
    g = D.all_gather(x)
    parts = [torch.empty(3, 5) for _ in range(WORLD)]
    dist.all_gather(parts, x.detach())
    assert torch.equal(g.detach(), torch.cat(parts, 0))
    # every rank's loss reads the whole gathered batch with its own weights;
    # d(sum of all ranks' losses)/dx_r = sum over ranks of their weight slice r
    w = torch.arange(WORLD * 15, dtype=torch.float32).reshape(WORLD * 3, 5) * (rank + 1)
    (g * w).sum().backward()
    wsum = torch.arange(WORLD * 15, dtype=torch.float32).reshape(WORLD * 3, 5) * sum(r + 1 for r in range(WORLD))
    assert torch.allclose(x.grad, wsum[rank * 3:(rank + 1) * 3])
    # non-differentiable path (lengths / class ids are int64 and must arrive bit-exact)
    ids = torch.tensor([7 + rank, 200 - rank], dtype=torch.int64)
    got = D.all_gather(ids, differentiable=False)
    assert got.tolist() == [7, 200, 8, 199]


def _case_flat_adam_allreduce(rank):
    from eegan_hip.optim import FlatAdam
    torch.manual_seed(7)
    ps = [torch.nn.Parameter(torch.randn(s)) for s in [(5, 3), (7,), (1,), (4, 4, 2)]]
    opt = FlatAdam(ps, lr=1e-3, betas=(0.0, 0.9), process_group=dist.group.WORLD, bucket_bytes=24)  # 6-float buckets
    torch.manual_seed(1000 + rank)
    local = [torch.randn(p.shape) for p in ps]
    for p, g in zip(ps, local):
        p.grad.copy_(g)
    opt._allreduce()
    allg = [torch.empty(opt.numel) for _ in range(WORLD)]
    dist.all_gather(allg, torch.cat([torch.cat([g.reshape(-1), torch.zeros((-g.numel()) % 4)]) for g in local]))
    mean = sum(allg) / WORLD
    assert torch.allclose(opt.gflat, mean, atol=1e-6)
    for p in ps:  # parameter .grad stays a view into the averaged flat buffer
        assert p.grad.data_ptr() >= opt.gflat.data_ptr()


def _case_flat_adam_overlap_plans(rank):
    """FlatAdam's overlapped all-reduce over learned write plans (the kernels'
    direct gradient writes simulated on CPU): two kinds of window share one
    key (same first parameter, same writing Function) but write parameters
    different numbers of times -- a first-order backward (one write each) and
    a double backward (two writes to some).  Each key's first two windows only
    learn; from then on a bucket is reduced during the backward only when
    every plan still consistent with the writes agrees it is complete; every
    window's result equals the mean over ranks, and buckets written from two
    streams wait for step()."""
    import types
    from eegan_hip import optim as OP
    torch.manual_seed(7)
    ps = [torch.nn.Parameter(torch.randn(8)) for _ in range(4)]
    opt = OP.FlatAdam(ps, lr=1e-3, betas=(0.0, 0.9), process_group=dist.group.WORLD, bucket_bytes=32)
    assert len(opt.buckets) == 4   # one parameter per bucket
    OP.ops = types.SimpleNamespace(fill_f32=lambda ptr, n, v, st: opt.gflat.fill_(v))
    OP.stream = lambda: 0
    early = []
    orig = opt._reduce_bucket
    opt._reduce_bucket = lambda b: (early.append((opt._in_bwd, b)), orig(b))[1]
    kinds = {'first': [3, 2, 1, 0], 'double': [3, 2, 2, 1, 1, 0]}
    g = torch.Generator().manual_seed(100 + rank)
    for it, kind in enumerate(['first', 'double'] * 3 + ['double', 'first']):
        early.clear()
        opt.zero_grad()
        local = torch.zeros(opt.numel)
        opt._in_bwd = True
        for i in kinds[kind]:
            v = torch.randn(8, generator=g)
            ps[i].grad.add_(v)
            local[opt._offs[i]:opt._offs[i] + 8] += v
            if opt.note_grad_write(ps[i], 'ConvFnBackward'):
                opt.flush_ready()
        opt._in_bwd = False
        opt._allreduce()
        allg = [torch.empty(opt.numel) for _ in range(WORLD)]
        dist.all_gather(allg, local)
        assert torch.allclose(opt.gflat, sum(allg) / WORLD, atol=1e-6), (it, kind)
        during = sorted(b for d, b in early if d)
        if it < 2:
            assert during == [], (it, during)    # learning windows
        elif kind == 'first':
            # bucket of parameter 3 (bucket 0): one write in both plans -> early;
            # parameters 2 and 1 were written once: the double plan wants two
            assert opt._bucket_of[3] in during and opt._bucket_of[2] not in during
        else:
            assert opt._bucket_of[3] in during and opt._bucket_of[2] in during, (it, during)
    # a bucket written from two streams is never reduced before step()
    opt.zero_grad()
    w = opt._win
    opt._in_bwd = True
    early.clear()
    for i in kinds['first']:
        if i == 3:
            w['streams'][opt._bucket_of[3]] = 12345   # an earlier write from another lane
        if opt.note_grad_write(ps[i], 'ConvFnBackward'):
            opt.flush_ready()
    opt._in_bwd = False
    assert opt._bucket_of[3] not in [b for d, b in early if d]
    opt._allreduce()


def _case_grad_reducer(rank):
    from eegan_hip.dist import GradReducer
    m = torch.nn.Linear(4, 3)
    for p in m.parameters():
        p.grad = torch.full_like(p, float(rank + 1))
    GradReducer(m).sync()
    for p in m.parameters():
        assert torch.allclose(p.grad, torch.full_like(p, (1 + WORLD) / 2.0))


def _case_grad_hooks_adam(rank):
    """GradHooks (installed by the drop-in models' forward) under an unchanged
    train.py loop: torch.optim.Adam, no explicit sync call.  Each rank's loss
    is the mean over its half of the batch; after backward + step on every
    rank the parameters equal one single-process step on the whole batch (the
    reference's nn.DataParallel semantics).  Includes a parameter that never
    receives a gradient (resD.conv_s when fin == fout), two backwards
    accumulated before one step, and small buckets so several all-reduces are
    in flight."""
    from eegan_hip import dist as D
    torch.manual_seed(3)

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a = torch.nn.Linear(6, 16)
            self.b = torch.nn.Linear(16, 4)
            self.unused = torch.nn.Linear(4, 4)

        def forward(self, x):
            return self.b(torch.relu(self.a(x)))

    net, ref = Net(), Net()
    ref.load_state_dict(net.state_dict())
    hooks = D.GradHooks(net, bucket_bytes=64)   # several buckets
    net._eegan_grad_hooks = hooks
    assert D.ensure_grad_hooks(net) is hooks and len(hooks.buckets) > 2
    opt = torch.optim.Adam(net.parameters(), lr=1e-2, betas=(0.0, 0.9))
    opt_r = torch.optim.Adam(ref.parameters(), lr=1e-2, betas=(0.0, 0.9))
    g = torch.Generator().manual_seed(11)
    for it in range(3):
        xs = [torch.randn(2 * WORLD, 6, generator=g) for _ in range(2)]
        opt.zero_grad()
        opt_r.zero_grad()
        for x in xs:   # two backwards accumulate before the step
            net(x[rank * 2:(rank + 1) * 2]).square().mean().backward()
            ref(x).square().mean().backward()
        for p, q in zip(net.parameters(), ref.parameters()):
            if q.grad is None:
                assert p.grad is None
            else:
                assert torch.allclose(p.grad, q.grad, atol=1e-6), it
        opt.step()
        opt_r.step()
    for p, q in zip(net.parameters(), ref.parameters()):
        assert torch.allclose(p, q, atol=1e-5)
    # FlatAdam-owned parameters are averaged by FlatAdam itself, never hooked
    m = torch.nn.Linear(3, 3)
    m.weight._eegan_gen = [0]
    h2 = D.GradHooks(m)
    assert all(p is not m.weight for b in h2.buckets for p in b)


def _case_syncbn_stats(rank):
    """Per-rank fp64 (sum, sumsq) -> all-reduce -> mean / clamp(var, eps)^-1/2
    on the global count, as the SyncBN Functions combine them across ranks,
    equals the oracle's multi-device BN on the concatenated batch."""
    from eegan_hip import dist as D
    from oracle import eegan_oracle as O
    D.install_syncbn_hook()
    from eegan_hip import functional as Fn
    assert Fn.SYNC_BN_WORLD == WORLD and Fn.SYNC_BN_ALLREDUCE is not None
    torch.manual_seed(55)
    full = torch.randn(2 * WORLD, 6, 5, 5) * 3 + 1
    full[:, 2] = 0.25  # constant channel: variance below eps exercises the clamp
    x = full[rank * 2:(rank + 1) * 2]
    sums = torch.cat([x.double().sum((0, 2, 3)), (x.double() ** 2).sum((0, 2, 3))])
    Fn.SYNC_BN_ALLREDUCE(sums)
    C = 6
    count = full.shape[0] * 25
    mean = sums[:C] / count
    var = (sums[C:] - sums[:C] * mean).clamp_min(0) / count
    istd = var.clamp_min(1e-5).rsqrt()
    y = (x.double() - mean.view(1, C, 1, 1)) * istd.view(1, C, 1, 1)
    sd = {'bn.weight': torch.ones(C), 'bn.bias': torch.zeros(C), 'bn.running_mean': torch.zeros(C),
          'bn.running_var': torch.ones(C)}
    ref = O.sync_bn(full, sd, 'bn.', affine=True, training=True, mode='multi')
    assert np.allclose(y.numpy(), ref[rank * 2:(rank + 1) * 2].detach().double().numpy(), atol=1e-5)
    # running statistics: unbiased variance of the global batch, momentum 0.1
    rv = 0.9 + 0.1 * var * count / (count - 1)
    assert torch.allclose(rv.float(), sd['bn.running_var'], atol=1e-5)


def _case_syncbn_peer_combine(rank):
    """EEGAN_SYNCBN_PEER's combine (eegan_hip.peer): every rank ends with the
    same bits, 0 + m_0 + ... + m_{W-1} in rank order (the peer kernel's sum),
    within fp64 rounding of the group's own all-reduce; the SyncBN hook routes
    through it when the switch is on."""
    from eegan_hip import dist as D
    from eegan_hip import functional as Fn
    from eegan_hip.peer import PeerAllReduce
    W = dist.get_world_size()
    assert not D.peer_syncbn()        # unset: on only for GPU ranks over RCCL, not for gloo
    D.PEER = '1'
    try:
        D.install_syncbn_hook()
        assert isinstance(Fn.SYNC_BN_ALLREDUCE, PeerAllReduce) and Fn.SYNC_BN_WORLD == W
        for n in (1, 7, 2 * 512):
            msgs = [torch.randn(n, dtype=torch.float64, generator=torch.Generator().manual_seed(1000 * r + n)) *
                    10.0 ** (r - 1) for r in range(W)]   # magnitudes differ: the order shows in the bits
            t = msgs[rank].clone()
            Fn.SYNC_BN_ALLREDUCE(t)
            want = torch.zeros(n, dtype=torch.float64)
            for m in msgs:
                want += m
            assert torch.equal(t, want)
            everyone = [torch.empty_like(t) for _ in range(W)]
            dist.all_gather(everyone, t)
            assert all(torch.equal(e, t) for e in everyone)
            ref = msgs[rank].clone()
            dist.all_reduce(ref)
            assert torch.allclose(t, ref, rtol=1e-14, atol=0)
    finally:
        D.PEER = None
        D.install_syncbn_hook()


def _case_peer_build_fallback_one_rank_fails(rank):
    """PeerAllReduce._build when only the last rank cannot map its peers'
    regions (peer_open failing there): every rank must agree on the fallback,
    no rank may block in a round the failing rank skips, and the ranks that
    did build a region close it after the closing exchange."""
    from eegan_hip import peer as P

    closed = []

    class FakeRegion(object):
        def __init__(self, group, cap):
            if dist.get_rank(group) == dist.get_world_size(group) - 1:
                raise RuntimeError('peer_open: simulated failure')

        def close(self):
            closed.append(True)

    real = P.PeerRegion
    P.PeerRegion = FakeRegion
    try:
        red = P.PeerAllReduce(group=dist.group.WORLD)
        import warnings
        with warnings.catch_warnings():
            warnings.simplefilter('ignore')
            assert red._build() is None
    finally:
        P.PeerRegion = real
    assert red.fallback is not None
    last = rank == dist.get_world_size() - 1
    assert closed == ([] if last else [True]), (rank, closed)
    # and the group is still in step: one more collective completes on every rank
    t = torch.ones(1)
    dist.all_reduce(t)
    assert float(t) == dist.get_world_size()


def test_gloo_world3_peer_build_fallback():
    _run(_case_peer_build_fallback_one_rank_fails, world=3)


def test_gloo_world3_syncbn_peer_combine():
    _run(_case_syncbn_peer_combine, world=3)


@pytest.mark.parametrize('case', ['syncbn_peer_combine', 'all_gather', 'flat_adam_allreduce', 'flat_adam_overlap_plans', 'grad_reducer', 'grad_hooks_adam', 'syncbn_stats'])
def test_gloo_world2(case):
    _run(globals()['_case_' + case])
