"""Data-parallel wrapper (API of sync_batchnorm/replicate.py).

The reference replicates the module onto every GPU inside ONE process each
forward (nn.DataParallel + replication callbacks, replicate.py:50-67).  Here
data parallelism is one process per GPU (torch.distributed over RCCL): the
wrapper keeps `.module` (train.py reaches COND_DNET through it), prefixes the
state_dict keys with `module.` like DataParallel, and -- when a process group
is up -- averages gradients across ranks with bucketed all-reduces launched
from post-accumulate-grad hooks (eegan_hip.dist.GradReducer)."""
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
    def __init__(self, module, device_ids=None, output_device=None, dim=0, grad_reduce=True):
        super().__init__()
        self.module = module
        self.device_ids = device_ids
        self.dim = dim
        self.reducer = None
        if grad_reduce:
            from eegan_hip import dist
            if dist.world_size() > 1:
                self.reducer = dist.GradReducer(module)

    def forward(self, *inputs, **kwargs):
        return self.module(*inputs, **kwargs)


DataParallel = DataParallelWithCallback


def patch_replication_callback(data_parallel):
    return data_parallel
