"""Data-parallel wrapper (API of sync_batchnorm/replicate.py).

The reference replicates the module onto every GPU inside ONE process each
forward (nn.DataParallel + replication callbacks, replicate.py:50-67).  Here
data parallelism is one process per GPU (torch.distributed over RCCL): the
wrapper keeps `.module` (train.py reaches COND_DNET through it) and prefixes
the state_dict keys with `module.` like DataParallel.  Gradient averaging is
not the wrapper's job: the drop-in models (models.Gen / ATTR_Enhance /
Dis64/128/256) install eegan_hip.dist.GradHooks on their first forward when a
process group with world > 1 is up -- bucketed all-reduces fired by
post-accumulate-grad hooks and flushed at the end of each backward -- so the
same averaging happens for D and ATTR_Enhance, which train.py wraps in
torch's own nn.DataParallel (train.py:222,228).  SyncBN statistics are
all-reduced inside the kernels' autograd Functions."""
import torch.nn as nn

__all__ = ['CallbackContext', 'execute_replication_callbacks', 'DataParallelWithCallback',
           'patch_replication_callback']


class CallbackContext(object):
    pass


def execute_replication_callbacks(modules):
    """Kept for API compatibility: one process owns one replica, nothing to wire."""
    master = modules[0]
    ctxs = [CallbackContext() for _ in master.modules()]
    for i, module in enumerate(modules):
        for j, m in enumerate(module.modules()):
            if hasattr(m, '__data_parallel_replicate__'):
                m.__data_parallel_replicate__(ctxs[j], i)


class DataParallelWithCallback(nn.Module):
    def __init__(self, module, device_ids=None, output_device=None, dim=0):
        super().__init__()
        self.module = module
        self.device_ids = device_ids
        self.dim = dim

    def forward(self, *inputs, **kwargs):
        return self.module(*inputs, **kwargs)


DataParallel = DataParallelWithCallback


def patch_replication_callback(data_parallel):
    return data_parallel
