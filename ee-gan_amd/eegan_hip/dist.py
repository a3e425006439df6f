"""Data-parallel plumbing: one process per GPU over torch.distributed
(backend "nccl" = RCCL on ROCm, "gloo" for CPU tests).

Replaces the single-process nn.DataParallel + host-thread SyncBN rendezvous
of the reference (train.py:220-228, its sync_batchnorm/comm.py) with:
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


# Rehearsal switch (EEGAN_FORCE_DIST=1): initialise a process group and issue
# every collective of the data-parallel step even with ONE rank, so the RCCL
# path (incl. its capture into the step's HIP graph) runs on a one-GPU box.
FORCE = os.environ.get('EEGAN_FORCE_DIST') == '1'
COMMS = []    # eegan_hip.rccl.Communicator per stream lane when the ranks own GPUs (graph-capturable)
# SyncBN statistics by the one-shot peer-write kernel (eegan_hip.peer) instead
# of RCCL: EEGAN_SYNCBN_PEER=1 / 0 forces it on / off; unset, it is on when the
# ranks own GPUs over RCCL (backend "nccl", world > 1).  The regions are
# validated collectively when they are built; if any rank cannot map or
# exchange through them, every rank keeps RCCL (eegan_hip.peer)
PEER = os.environ.get('EEGAN_SYNCBN_PEER')
N_LANES = 7   # lane 0: the caller's (main) stream; 1..: streams bound with bind_stream
_LANE_OF = {}


def bind_stream(stream, lane):
    """Collectives issued on `stream` use communicator `lane + 1` (lane >= 0)."""
    if lane + 1 >= N_LANES:
        raise ValueError('eegan_hip.dist: only %d stream lanes' % (N_LANES - 1))
    _LANE_OF[stream.cuda_stream] = lane + 1


def comm():
    """The RCCL communicator of the current stream's lane (None without GPU ranks)."""
    if not COMMS:
        return None
    return COMMS[_LANE_OF.get(torch.cuda.current_stream().cuda_stream, 0)]


def is_on():
    return dist.is_available() and dist.is_initialized()


def world_size():
    return dist.get_world_size() if is_on() else 1


def rank():
    return dist.get_rank() if is_on() else 0


def collective():
    """True when the step must issue its collectives (world > 1, or forced)."""
    return is_on() and (world_size() > 1 or FORCE)


def init_from_env(backend=None):
    """Initialise from torchrun's env (RANK/WORLD_SIZE/MASTER_ADDR/MASTER_PORT)."""
    ws = int(os.environ.get('WORLD_SIZE', '1'))
    if (ws <= 1 and not FORCE) or is_on():
        if is_on() and dist.get_backend() == 'nccl' and not COMMS and \
                os.environ.get('EEGAN_OWN_RCCL', '1') == '1':
            # a group started at import (eegan_hip.launch) or by the caller
            from .rccl import Communicator
            COMMS[:] = [Communicator(torch.cuda.current_device()) for _ in range(N_LANES)]
        install_syncbn_hook()
        return rank(), world_size()
    if backend is None:
        backend = os.environ.get('EEGAN_DIST_BACKEND') or ('nccl' if torch.cuda.is_available() else 'gloo')
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29561')
    os.environ.setdefault('RANK', '0')
    os.environ.setdefault('WORLD_SIZE', '1')
    dist.init_process_group(backend=backend)
    if backend == 'nccl' and os.environ.get('EEGAN_OWN_RCCL', '1') == '1':
        from .rccl import Communicator
        COMMS[:] = [Communicator(torch.cuda.current_device()) for _ in range(N_LANES)]
    install_syncbn_hook()
    return rank(), world_size()


def peer_syncbn(group=None):
    """Whether SyncBN statistics go through the peer-write all-reduce."""
    if PEER is not None:
        return PEER == '1'
    return is_on() and dist.get_backend(group) == 'nccl' and dist.get_world_size(group) > 1


def install_syncbn_hook(group=None):
    if is_on() and (dist.get_world_size(group) > 1 or FORCE):
        if peer_syncbn(group):
            from .peer import PeerAllReduce
            Fn.SYNC_BN_ALLREDUCE = PeerAllReduce(group)
        elif COMMS and group is None:
            Fn.SYNC_BN_ALLREDUCE = all_reduce
        else:
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
        ctx.n = x.shape[0]
        ctx.r = rank()
        return _gather(x)

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        all_reduce(g)
        return g[ctx.r * ctx.n:(ctx.r + 1) * ctx.n]


def all_reduce(t):
    """In-place sum over ranks (own RCCL communicator for device tensors)."""
    c = comm() if t.is_cuda and t.is_contiguous() else None
    if c is not None:
        c.all_reduce(t)
    else:
        dist.all_reduce(t)


def broadcast(t, src=0):
    """In place: rank `src`'s t on every rank (own RCCL communicator for device tensors)."""
    c = comm() if t.is_cuda and t.is_contiguous() else None
    if c is not None:
        c.broadcast(t, src)
    else:
        dist.broadcast(t, src)


def all_gather_bytes(b, device=None):
    """[every rank's b] (equal lengths): over the current lane's own RCCL
    communicator when the ranks own GPUs (no ProcessGroupNCCL work that its
    watchdog would still track when a graph capture starts), else through the
    process group.  Synchronises the host."""
    if COMMS:
        x = torch.tensor(list(b), dtype=torch.uint8, device=device if device is not None else 'cuda')
        out = _gather(x).cpu().reshape(world_size(), len(b))
        return [bytes(row.tolist()) for row in out]
    out = [None] * world_size()
    dist.all_gather_object(out, bytes(b))
    return out


def _gather(x):
    c = comm() if x.is_cuda else None
    if c is not None:
        return c.all_gather(x)
    out = [torch.empty_like(x) for _ in range(world_size())]
    dist.all_gather(out, x)
    return torch.cat(out, 0)


def all_gather(x, differentiable=True):
    if not collective():
        return x
    if differentiable and x.requires_grad:
        return AllGatherFn.apply(x)
    return _gather(x.contiguous())


class GradReducer(object):
    """Explicit gradient averaging: averages every parameter's .grad across
    ranks when `sync()` is called.  Kept for callers that drive the reduction
    themselves; the drop-in modules average through GradHooks instead."""

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


class GradHooks(object):
    """Gradient averaging across ranks for an unchanged reference train.py
    (torch.optim.Adam, train.py:252-263): the reference's single-process
    nn.DataParallel reduce-adds replica gradients to GPU0 inside every
    backward (train.py:220-228); here each parameter of the module gets a
    post-accumulate-grad hook, parameters are grouped into buckets in reverse
    registration order (roughly the order backward produces them), a bucket's
    flattened gradients are all-reduced asynchronously as soon as all of its
    members have accumulated, and an end-of-backward callback flushes the
    partial buckets (parameters that got no gradient in this backward, e.g.
    resD.conv_s when fin == fout, are skipped -- every rank runs the same graph,
    so the skipped set agrees), waits, divides by the world size and writes the
    averages back into .grad.

    Averaging the accumulated .grad is exact even when a backward adds to a
    gradient that an earlier backward already averaged: that earlier part is
    identical on every rank, and the mean is linear.  Parameters owned by a
    FlatAdam (eegan_hip.optim) are skipped: it averages its flat buffer
    itself.  Parameters are flagged `_eegan_hooked`, which turns off the
    kernels' direct accumulation into .grad for them (that path bypasses
    AccumulateGrad, whose hooks this relies on)."""

    def __init__(self, module, bucket_bytes=25 << 20):
        params = [p for p in module.parameters() if p.requires_grad and not hasattr(p, '_eegan_gen')]
        self.buckets = []
        cur, size = [], 0
        for p in reversed(params):
            if getattr(p, '_eegan_hooked', False):
                continue  # shared with another hooked module
            cur.append(p)
            size += p.numel() * p.element_size()
            if size >= bucket_bytes:
                self.buckets.append(cur)
                cur, size = [], 0
        if cur:
            self.buckets.append(cur)
        self._where = {}
        for bi, b in enumerate(self.buckets):
            for p in b:
                p._eegan_hooked = True
                self._where[id(p)] = bi
                p.register_post_accumulate_grad_hook(self._hook)
        self._reset()

    def _reset(self):
        self._fired = [[] for _ in self.buckets]
        self._works = []
        self._queued = False

    def _launch(self, bi):
        ps = self._fired[bi]
        if not ps:
            return
        flat = torch.cat([p.grad.reshape(-1) for p in ps])
        work = dist.all_reduce(flat, async_op=True)
        self._works.append((work, flat, list(ps)))
        self._fired[bi] = None   # launched

    def _hook(self, p):
        if not collective() or getattr(p, '_eegan_gen', None) is not None:
            return
        bi = self._where[id(p)]
        if self._fired[bi] is None:    # a second backward over an already-reduced bucket: start over
            self._fired[bi] = []
        self._fired[bi].append(p)
        if len(self._fired[bi]) == len(self.buckets[bi]):
            self._launch(bi)
        if not self._queued:
            self._queued = True
            torch.autograd.Variable._execution_engine.queue_callback(self._finish)

    def _finish(self):
        self._backwards = getattr(self, '_backwards', 0) + 1
        if self._backwards % CHECK_EVERY == 0:
            check_collectives()
        for bi in range(len(self.buckets)):
            if self._fired[bi]:
                self._launch(bi)
        inv = 1.0 / world_size()
        for work, flat, ps in self._works:
            work.wait()
            flat.mul_(inv)
            o = 0
            for p in ps:
                n = p.grad.numel()
                p.grad.copy_(flat[o:o + n].view_as(p.grad))
                o += n
        self._reset()


def broadcast_state(module, src=0):
    """Rank `src`'s parameters and buffers into every rank's module, in place
    (torch DDP does this when it wraps a module).  Under an unchanged train.py
    the ranks build their models after eegan_hip.launch.offset_rank_rngs gave
    each rank its own random streams, so their initial weights differ; the
    reference's replicas all start from GPU0's module (train.py:220-228)."""
    with torch.no_grad():
        for t in list(module.parameters()) + list(module.buffers()):
            x = t.data
            if not x.is_contiguous() and x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last):
                x = x.permute(0, 2, 3, 1)   # channels-last conv weights: a contiguous view of the storage
            if not x.is_contiguous():
                raise RuntimeError('eegan_hip: cannot broadcast a non-dense %s of shape %s'
                                   % (type(module).__name__, tuple(t.shape)))
            broadcast(x, src)


def check_collectives():
    """Raise if a SyncBN peer-write reduction timed out (EEGAN_SYNCBN_PEER;
    csrc/peer.hip poisons its output with NaN and every later call of that
    lane at once).  Synchronises the device when the peer path is on; a no-op
    otherwise.  Called by the trainer every CHECK_EVERY steps, by GradHooks
    every CHECK_EVERY backwards (an unchanged train.py) and before any drop-in
    model's state_dict is taken (a desynchronised rank must not write a
    checkpoint, train.py:310-318)."""
    red = Fn.SYNC_BN_ALLREDUCE
    if red is not None and hasattr(red, 'check'):
        red.check()


CHECK_EVERY = 64   # steps (or backwards) between the periodic checks above


def guard_state_dict(module):
    """state_dict() of `module` (and of any wrapper around it: torch's
    state_dict recurses through the children's state_dict) checks the
    collectives first."""
    module.register_state_dict_pre_hook(lambda m, prefix, keep_vars: check_collectives())


def ensure_grad_hooks(module):
    """Install GradHooks on `module` once, when the step is data-parallel
    (called from the drop-in models' forward, so reference code that wraps D
    and ATTR_Enhance in torch's own nn.DataParallel gets them too)."""
    if getattr(module, '_eegan_grad_hooks', None) is None:
        from .launch import check_process_group
        check_process_group()   # torchrun ranks without a process group: refuse to train alone
    if getattr(module, '_eegan_grad_hooks', None) is None and collective():
        if any(p.requires_grad and not p.is_leaf for p in module.parameters()):
            # torch's nn.DataParallel replicated the module over several visible
            # GPUs: its parameters are non-leaf copies (no post-accumulate hook
            # possible) and the original parameters would never be averaged
            raise RuntimeError('eegan_hip: %s runs as an nn.DataParallel replica (non-leaf parameters); the '
                               'data-parallel drop-in needs ONE visible GPU per rank (CUDA_VISIBLE_DEVICES / '
                               'HIP_VISIBLE_DEVICES set per rank, see INTEGRATION.md)' % type(module).__name__)
        broadcast_state(module)
        module._eegan_grad_hooks = GradHooks(module)
    return getattr(module, '_eegan_grad_hooks', None)
