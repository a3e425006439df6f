"""One rank of the SyncBN peer-write all-reduce check (eegan_hip.peer,
csrc/peer.hip), launched by tests/test_gpu_peer.py as two torchrun ranks that
share one GPU (gloo group for the IPC handle exchange).  Writes OUT/peerR.pt:
the reduced messages (eager, and from replays of a captured graph), the
fixed-order host sums they must equal, SyncBN outputs / input gradients with
the peer path and with the group's all-reduce, the kernel's timeout flag and
its latency per call."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in (REPO, os.path.join(REPO, 'ee-gan_amd'), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def msg(r, n, k):
    g = torch.Generator().manual_seed(7919 * r + 31 * n + k)
    return torch.randn(n, dtype=torch.float64, generator=g) * 10.0 ** (r - 1)


def host_sum(W, n, k):
    acc = torch.zeros(n, dtype=torch.float64)
    for r in range(W):
        acc += msg(r, n, k)
    return acc


def main(out):
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    dist.init_process_group('gloo')
    rank, W = dist.get_rank(), dist.get_world_size()
    from eegan_hip.peer import PeerAllReduce
    red = PeerAllReduce()
    res = {'eager': [], 'graph': []}
    # eager calls, several sizes (up to the region capacity)
    for k, n in enumerate((1, 7, 1024, 4096)):
        t = msg(rank, n, k).to(dev)
        red(t)
        torch.cuda.synchronize()
        res['eager'].append((t.cpu(), host_sum(W, n, k)))
        if red.timed_out():
            raise SystemExit('peer wait timed out at n=%d' % n)
    # captured: three calls on a side stream, replayed with fresh contents
    side = torch.cuda.Stream()
    bufs = [torch.zeros(n, dtype=torch.float64, device=dev) for n in (16, 300, 2048)]
    with torch.cuda.stream(side):
        for b in bufs:
            red(b)   # eager first call on this stream creates its region
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        for b in bufs:
            red(b)
    for rep in range(4):
        for i, b in enumerate(bufs):
            b.copy_(msg(rank, b.numel(), 100 + 10 * rep + i))
        dist.barrier()
        g.replay()
        torch.cuda.synchronize()
        res['graph'].append([(b.cpu(), host_sum(W, b.numel(), 100 + 10 * rep + i)) for i, b in enumerate(bufs)])
    # SyncBN through the peer path vs the group's all-reduce (bit-identical at 2 ranks: a + b either way)
    from eegan_hip import functional as Fn
    from sync_batchnorm import SynchronizedBatchNorm2d
    torch.manual_seed(3)
    x = (torch.randn(2 * W, 40, 9, 9) * 2 + 0.5)[2 * rank:2 * rank + 2].to(dev)
    rgrad = torch.randn(2 * W, 40, 9, 9)[2 * rank:2 * rank + 2].to(dev)
    outs = {}
    for tag, fn in (('peer', red), ('group', lambda t: dist.all_reduce(t))):
        Fn.SYNC_BN_ALLREDUCE, Fn.SYNC_BN_WORLD = fn, W
        bn = SynchronizedBatchNorm2d(40).to(dev)
        xd = x.clone().requires_grad_()
        y = bn(xd)
        (y.float() * rgrad).sum().backward()
        torch.cuda.synchronize()
        outs[tag] = (y.float().cpu(), xd.grad.cpu(), bn.running_var.cpu())
    res['bn'] = outs
    # latency per call (eager, 8 KB message), both ranks issuing together
    t = msg(rank, 1024, 0).to(dev)
    dist.barrier()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(200):
        red(t)
    e1.record()
    torch.cuda.synchronize()
    res['us_per_call'] = e0.elapsed_time(e1) * 1e3 / 200
    res['timed_out'] = red.timed_out()
    dist.barrier()
    red.close()
    torch.save(res, os.path.join(out, 'peer%d.pt' % rank))
    dist.destroy_process_group()


if __name__ == '__main__':
    main(sys.argv[1])
