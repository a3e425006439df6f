from .batchnorm import SynchronizedBatchNorm1d, SynchronizedBatchNorm2d, SynchronizedBatchNorm3d
from .replicate import (CallbackContext, DataParallelWithCallback, RankGroup, execute_replication_callbacks,
                        patch_replication_callback)
