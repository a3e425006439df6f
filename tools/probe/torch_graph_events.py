"""Probe: external event records (via libeegan_hip) inside torch.cuda.graph captures."""
import ctypes
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..', 'ee-gan_amd'))
import torch  # noqa: E402
from eegan_hip._lib import ops  # noqa: E402
from eegan_hip.tensor import stream  # noqa: E402

x = torch.randn(1 << 22, device='cuda')
for mode in ('global', 'thread_local', 'relaxed'):
    e0, e1 = ctypes.c_void_p(), ctypes.c_void_p()
    ops.event_create(ctypes.byref(e0))
    ops.event_create(ctypes.byref(e1))
    g = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(g, capture_error_mode=mode):
            ops.event_record(e0, stream())
            y = x * 2 + 1
            ops.event_record(e1, stream())
        g.replay()
        torch.cuda.synchronize()
        ms = ctypes.c_float()
        ops.event_elapsed(e0, e1, ctypes.byref(ms))
        print(mode, 'ok', ms.value)
    except Exception as ex:
        print(mode, 'FAILED', ex)
