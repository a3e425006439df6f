"""eegan_hip: host glue of the MI355X EE-GAN training step.

libeegan_hip.so (ee-gan_amd/csrc, C ABI in include/eegan_hip.h) holds every
kernel; this package binds it with ctypes (_lib), wraps the kernels as
autograd Functions (functional), provides the parameter modules (nn), the
flat fused Adam (optim), the data-parallel plumbing (dist) and the inner
training step (trainer).  Importing it fails loudly when the library is
missing -- there is no CPU/PyTorch fallback.
"""
from . import launch as _launch

# under torchrun with WORLD_SIZE > 1: pin this rank's GPU and join the ranks
# before anything starts the HIP runtime (an unchanged reference train.py
# never does either; eegan_hip.launch)
_launch.setup()

from ._lib import LIB, ABI_VERSION, ops, exported_symbols  # noqa: F401,E402

__all__ = ['LIB', 'ABI_VERSION', 'ops', 'exported_symbols']
