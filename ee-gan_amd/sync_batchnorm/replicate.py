"""Data-parallel wrapper: the API of the reference's sync_batchnorm/replicate.py
(CallbackContext, execute_replication_callbacks, DataParallelWithCallback,
patch_replication_callback; replicate.py:23-88).

The reference replicates the module onto every GPU inside ONE process at each
forward and wires the SyncBN replicas together through replication callbacks
(`__data_parallel_replicate__(ctx, copy_id)`: copy 0 becomes the SyncMaster,
the others register slave pipes with it).  Here data parallelism is one
process per GPU (torch.distributed over RCCL, eegan_hip.launch /
eegan_hip.dist): every rank holds the ONE copy it runs, so the replication
step happens once, when the module is wrapped, with copy_id = the rank.  The
callbacks then see what the reference's replicas see: `_is_parallel` (more
than one copy -- the reference's switch from F.batch_norm to the synchronised
statistics, batchnorm.py:50), `_parallel_id` (0 on the master copy) and a
context shared by all copies of one submodule, whose `sync_master` is the
rank group that carries the statistics exchange (eegan_hip.dist: RCCL or the
peer-write kernel) instead of SyncMaster's queues.

What DataParallel's forward does per call -- scatter the batch, broadcast the
master weights, gather the outputs, reduce the gradients -- is spread over
the ranks: each rank loads its own shard (datasets.TextDataset), rank 0's
weights are broadcast at the first forward and gradients are averaged by
eegan_hip.dist.GradHooks (installed by the drop-in models' forward), so the
wrapper keeps `.module` (train.py reaches COND_DNET through it), the `module.`
prefix of the state_dict keys, and forwards."""
import torch
import torch.nn as nn

__all__ = ['CallbackContext', 'execute_replication_callbacks', 'DataParallelWithCallback',
           'patch_replication_callback', 'RankGroup']


class CallbackContext(object):
    """Shared by all copies of one submodule (replicate.py:23-24)."""
    pass


class RankGroup(object):
    """The `sync_master` of a context: the process group over which the copies
    of one SyncBN layer exchange their statistics (the reference's SyncMaster,
    comm.py:18-137, without the queues: every rank reduces for itself)."""

    def __init__(self, world, rank, transport):
        self.world, self.rank, self.transport = world, rank, transport

    def __repr__(self):
        return 'RankGroup(world=%d, rank=%d, transport=%s)' % (self.world, self.rank, self.transport)


def _rank_world():
    from eegan_hip import dist as D
    return D.rank(), D.world_size()


def _transport():
    from eegan_hip import dist as D
    from eegan_hip import functional as Fn
    if not D.is_on() or Fn.SYNC_BN_ALLREDUCE is None:
        return 'local'
    return 'peer-write' if type(Fn.SYNC_BN_ALLREDUCE).__name__ == 'PeerAllReduce' else 'rccl'


def execute_replication_callbacks(modules, copy_ids=None):
    """Call `__data_parallel_replicate__(ctx, copy_id)` on every submodule of
    the given copies that defines it, one shared context per submodule
    position, the master copy (id 0) first (replicate.py:27-47).  One process
    per GPU passes its own copy with copy_ids=[rank]; the master's context
    gets the rank group, which every copy reads as ctx.sync_master."""
    if copy_ids is None:
        copy_ids = list(range(len(modules)))
    order = sorted(range(len(modules)), key=lambda i: copy_ids[i])
    master = modules[order[0]]
    ctxs = [CallbackContext() for _ in master.modules()]
    rank, world = _rank_world()
    for c in ctxs:
        c.sync_master = RankGroup(world, rank, _transport())
    for i in order:
        for j, m in enumerate(modules[i].modules()):
            if hasattr(m, '__data_parallel_replicate__'):
                m.__data_parallel_replicate__(ctxs[j], copy_ids[i])
    return ctxs


class DataParallelWithCallback(nn.Module):
    """replicate.py:50-67 for one process per GPU: the rank's copy is
    "replicated" once at wrap time (execute_replication_callbacks with
    copy_id = rank).  device_ids keeps the reference's meaning as the GPUs of
    the job; with torchrun each rank's process sees its own device first."""

    def __init__(self, module, device_ids=None, output_device=None, dim=0):
        super().__init__()
        self.module = module
        self.device_ids = list(device_ids) if device_ids is not None else None
        self.output_device = output_device
        self.dim = dim
        rank, _ = _rank_world()
        execute_replication_callbacks([module], [rank])

    def forward(self, *inputs, **kwargs):
        return self.module(*inputs, **kwargs)

    def replicate(self, module, device_ids):
        """The reference's override (replicate.py:63-67) on one device: the
        callbacks run on this rank's copy, which is returned as the only
        replica."""
        rank, _ = _rank_world()
        execute_replication_callbacks([module], [rank])
        return [module]


def patch_replication_callback(data_parallel):
    """replicate.py:70-88: make an existing nn.DataParallel run the
    replication callbacks.  One process per GPU: its module is replicated once,
    here, with copy_id = the rank (train.py wraps D and ATTR_Enhance in plain
    nn.DataParallel, whose single-device forward never replicates)."""
    assert isinstance(data_parallel, (torch.nn.DataParallel, DataParallelWithCallback))
    rank, _ = _rank_world()
    execute_replication_callbacks([data_parallel.module], [rank])
    return data_parallel
