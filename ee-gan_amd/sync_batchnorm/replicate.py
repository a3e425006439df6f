"""Data-parallel wrapper: the API of the reference's sync_batchnorm/replicate.py
(DataParallelWithCallback, patch_replication_callback; replicate.py:50-67).

The reference replicates the module onto every GPU inside ONE process each
forward and wires the SyncBN replicas together with replication callbacks.
Here data parallelism is one process per GPU (torch.distributed over RCCL,
eegan_hip.launch / eegan_hip.dist), so there are no replicas to wire: the
wrapper keeps `.module` (train.py reaches COND_DNET through it) and the
`module.` prefix of the state_dict keys, and forwards.  Gradient averaging
(eegan_hip.dist.GradHooks, installed by the drop-in models' forward) and the
SyncBN statistics all-reduce (inside the kernels' autograd Functions) happen
in the modules themselves, so they also cover D and ATTR_Enhance, which
train.py wraps in torch's own nn.DataParallel (train.py:222,228)."""
import torch.nn as nn

__all__ = ['DataParallelWithCallback', 'patch_replication_callback']


class DataParallelWithCallback(nn.Module):
    def __init__(self, module, device_ids=None, output_device=None, dim=0):
        super().__init__()
        self.module = module
        self.device_ids = device_ids
        self.dim = dim

    def forward(self, *inputs, **kwargs):
        return self.module(*inputs, **kwargs)


def patch_replication_callback(data_parallel):
    """replicate.py:70-88 patches an nn.DataParallel's replicate(); one process
    per GPU has nothing to patch."""
    return data_parallel
