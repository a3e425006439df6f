"""Data-parallel plumbing: one process per GPU over torch.distributed
(backend "nccl" = RCCL on ROCm, "gloo" for CPU tests).

Replaces the single-process nn.DataParallel + host-thread SyncBN rendezvous
of the reference (train.py:220-228, sync_batchnorm/comm.py) with:
  * SyncBN statistics all-reduce: a 2C-value fp64 message per BN layer in
    forward (sum, sumsq) and backward (sum dxhat, sum dxhat*xhat);
  * gradient averaging: bucketed all-reduce of each optimizer's flat gradient
    buffer (eegan_hip.optim.FlatAdam);
  * global-batch DAMSM: differentiable all-gather of image regions / codes
    and all-gather of text embeddings, lengths and class ids, so the
    contrastive B_global x B_global similarity matches the reference's
    DataParallel semantics (DAMSM_losses.py:233-342 over the gathered batch).
"""
import os

import torch
import torch.distributed as dist

from . import functional as Fn


def is_on():
    return dist.is_available() and dist.is_initialized()


def world_size():
    return dist.get_world_size() if is_on() else 1


def rank():
    return dist.get_rank() if is_on() else 0


def init_from_env(backend=None):
    """Initialise from torchrun's env (RANK/WORLD_SIZE/MASTER_ADDR/MASTER_PORT)."""
    ws = int(os.environ.get('WORLD_SIZE', '1'))
    if ws <= 1 or is_on():
        install_syncbn_hook()
        return rank(), world_size()
    if backend is None:
        backend = os.environ.get('EEGAN_DIST_BACKEND') or ('nccl' if torch.cuda.is_available() else 'gloo')
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    dist.init_process_group(backend=backend)
    install_syncbn_hook()
    return rank(), world_size()


def install_syncbn_hook(group=None):
    if is_on() and dist.get_world_size(group) > 1:
        Fn.SYNC_BN_ALLREDUCE = lambda t: dist.all_reduce(t, group=group)
        Fn.SYNC_BN_WORLD = dist.get_world_size(group)
    else:
        Fn.SYNC_BN_ALLREDUCE = None
        Fn.SYNC_BN_WORLD = 1


class AllGatherFn(torch.autograd.Function):
    """Differentiable all-gather along dim 0 (equal shards); backward = the
    rank's slice of the all-reduced gradient (a reduce-scatter)."""

    @staticmethod
    def forward(ctx, x):
        ws = world_size()
        x = x.contiguous()
        out = [torch.empty_like(x) for _ in range(ws)]
        dist.all_gather(out, x)
        ctx.n = x.shape[0]
        ctx.r = rank()
        return torch.cat(out, 0)

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        dist.all_reduce(g)
        return g[ctx.r * ctx.n:(ctx.r + 1) * ctx.n]


def all_gather(x, differentiable=True):
    if world_size() == 1:
        return x
    if differentiable and x.requires_grad:
        return AllGatherFn.apply(x)
    out = [torch.empty_like(x.contiguous()) for _ in range(world_size())]
    dist.all_gather(out, x.contiguous())
    return torch.cat(out, 0)


class GradReducer(object):
    """Gradient averaging for DataParallelWithCallback when the caller keeps
    torch.optim.Adam (reference train.py unchanged): averages every
    parameter's .grad across ranks when `sync()` is called (FlatAdam does this
    itself inside step())."""

    def __init__(self, module):
        self.params = [p for p in module.parameters() if p.requires_grad]

    def sync(self):
        if world_size() == 1:
            return
        grads = [p.grad for p in self.params if p.grad is not None]
        if not grads:
            return
        flat = torch.cat([g.reshape(-1) for g in grads])
        dist.all_reduce(flat)
        flat.mul_(1.0 / world_size())
        o = 0
        for g in grads:
            n = g.numel()
            g.copy_(flat[o:o + n].view_as(g))
            o += n
