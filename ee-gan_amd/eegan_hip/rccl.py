"""RCCL communicators of our own on the RCCL library torch already loaded.

The step's collectives (SyncBN statistics, DAMSM gathers, gradient buckets)
are issued as plain RCCL calls on the caller's HIP stream, so the whole
data-parallel step -- collectives included -- can be captured into the step's
HIP graph.  torch's ProcessGroupNCCL is used only to exchange the unique ids
and for host-side barriers outside the timed region: collectives it issues
inside a graph capture leave events its watchdog thread later queries, which
the HIP runtime rejects (hipErrorCapturedEvent) and aborts the process -- and
so does one issued just before a capture, while the watchdog still tracks it.
Set-up exchanges that run at a step's first (eager) pass -- the weight
broadcast of eegan_hip.dist.broadcast_state, the peer-region handles of
eegan_hip.peer -- therefore go over these communicators too.

Ordering: RCCL needs the operations of one communicator issued in the same
order on every rank and never concurrently from two streams.  The step runs
the three D updates (and the DAMSM branch) on their own streams, so each
stream lane gets its own communicator (eegan_hip.dist binds lanes to
streams); within a lane the program order is the issue order.  (Funnelling
every lane through one shared stream instead crashes hipStreamEndCapture on
this runtime: tools/probe/stream_probe.py.)
"""
import ctypes as C
import glob
import os

import torch

_DT = {torch.float32: 7, torch.float64: 8, torch.bfloat16: 9, torch.float16: 6, torch.int64: 4, torch.int32: 2,
       torch.uint8: 1, torch.int8: 0}
_SUM = 0


class _UniqueId(C.Structure):
    _fields_ = [('internal', C.c_ubyte * 128)]


def _load():
    cands = sorted(glob.glob(os.path.join(os.path.dirname(torch.__file__), 'lib', 'librccl*.so*')))
    if not cands:
        raise ImportError('RCCL library not found next to torch')
    lib = C.CDLL(cands[0], mode=C.RTLD_GLOBAL)
    lib.ncclGetUniqueId.argtypes = [C.POINTER(_UniqueId)]
    lib.ncclCommInitRank.argtypes = [C.POINTER(C.c_void_p), C.c_int, _UniqueId, C.c_int]
    lib.ncclAllReduce.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
    lib.ncclAllGather.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p, C.c_void_p]
    lib.ncclBroadcast.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
    lib.ncclCommDestroy.argtypes = [C.c_void_p]
    lib.ncclGetErrorString.restype = C.c_char_p
    lib.ncclGetErrorString.argtypes = [C.c_int]
    return lib


class Communicator(object):
    """RCCL communicator over the ranks of the default torch process group."""

    def __init__(self, device):
        import torch.distributed as dist
        self.lib = _load()
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        uid = _UniqueId()
        if self.rank == 0:
            self._check(self.lib.ncclGetUniqueId(C.byref(uid)), 'ncclGetUniqueId')
        box = [C.string_at(C.addressof(uid), 128) if self.rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        uid = _UniqueId()
        C.memmove(C.addressof(uid), box[0], 128)
        self.comm = C.c_void_p()
        with torch.cuda.device(device):
            self._check(self.lib.ncclCommInitRank(C.byref(self.comm), self.world, uid, self.rank), 'ncclCommInitRank')

    def _check(self, rc, what):
        if rc != 0:
            raise RuntimeError('%s failed (%d): %s' % (what, rc, self.lib.ncclGetErrorString(rc).decode()))

    def _run(self, fn):
        fn(torch.cuda.current_stream().cuda_stream)

    def all_reduce(self, t):
        """In-place sum over ranks of a contiguous device tensor."""
        assert t.is_contiguous() and t.is_cuda
        self._run(lambda s: self._check(self.lib.ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), _DT[t.dtype],
                                                               _SUM, self.comm, s), 'ncclAllReduce'))

    def all_gather(self, x):
        """Concatenation along dim 0 of every rank's x (equal shapes)."""
        x = x.contiguous()
        out = torch.empty((self.world * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        self._run(lambda s: self._check(self.lib.ncclAllGather(x.data_ptr(), out.data_ptr(), x.numel(), _DT[x.dtype],
                                                               self.comm, s), 'ncclAllGather'))
        return out

    def broadcast(self, t, root=0):
        """Rank `root`'s t into every rank's t (contiguous device tensor, in place)."""
        assert t.is_contiguous() and t.is_cuda
        self._run(lambda s: self._check(self.lib.ncclBroadcast(t.data_ptr(), t.data_ptr(), t.numel(), _DT[t.dtype],
                                                               root, self.comm, s), 'ncclBroadcast'))

    def close(self):
        if self.comm:
            self.lib.ncclCommDestroy(self.comm)
            self.comm = C.c_void_p()
