"""One-shot peer-write all-reduce for the SyncBN statistics (EEGAN_SYNCBN_PEER=1).

The reference exchanges every BN layer's (sum, ssum) message through a master
replica (reference sync_batchnorm/batchnorm.py:90-111 over SyncMaster / SlavePipe,
reference sync_batchnorm/comm.py:18-137): gather to GPU0, reduce, broadcast back.  With
one process per GPU these messages (2C fp64 values, at most a few KB) are
latency-bound; a ring all-reduce spends most of its time in protocol steps.
Here each rank owns a small uncached device region per stream lane, mapped by
every peer over IPC (xGMI between MI355X GPUs), and one kernel per call
(csrc/peer.hip) stores the rank's message into every rank's region, raises a
flag there, waits for all flags in its own region, and sums the slots in rank
order -- every rank gets identical bits, with no second hop.  The epoch
counter lives on the device, so the calls are graph-capturable and replay
correctly.

Regions are created collectively (the 64-byte IPC handles are exchanged with
all_gather_object over the process group) the first time a stream issues a
reduction, which must happen outside graph capture -- the trainer's eager
warm-up steps do it.  Messages longer than the region capacity go to the
group's regular all-reduce; host tensors (CPU process groups) take
`fixed_order_sum`.

`fixed_order_sum` is the combine's host restatement for CPU process groups
(the gloo tests): all-gather, then 0 + m_0 + ... + m_{W-1} in fp64.
"""
import ctypes as C
import os

import torch
import torch.distributed as dist

from ._lib import LIB, ops

MAX_RANKS = 16
CAP = 4096   # doubles per message: SyncBN sends 2C values, C <= 2048
# how long a reduction waits for a peer's slice before it gives up, poisons its
# result with NaN and sets the region's error word (Trainer.check_collectives then
# raises within CHECK_EVERY steps, which ends the run).  Host-side skew beyond
# this -- a rank writing a checkpoint, DataLoader workers respawning at an epoch
# boundary while the others already wait in their next SyncBN call -- is
# indistinguishable from a dead peer, so size it above the longest expected
# stall (EEGAN_PEER_WAIT_S, seconds; RCCL itself waits without bound)
WAIT_S = int(os.environ.get('EEGAN_PEER_WAIT_S', '30'))


class PeerRegion(object):
    """This rank's region for one stream lane plus the mapped regions of its peers."""

    def __init__(self, group=None, cap=CAP, device=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if self.world > MAX_RANKS:
            raise ValueError('eegan_hip.peer: at most %d ranks (got %d)' % (MAX_RANKS, self.world))
        self.cap = cap
        nbytes = LIB.eegan_peer_region_bytes(cap)
        own = C.c_void_p()
        handle = (C.c_ubyte * 64)()
        self.own, err = None, None
        try:
            with torch.cuda.device(device if device is not None else torch.cuda.current_device()):
                ops.peer_alloc(nbytes, C.byref(own), handle)
            self.own = own.value
            ops.peer_set_wait(self.own, WAIT_S)
        except Exception as e:
            err = str(e)
        self._opened = []
        # every rank joins the exchange, a failed allocation included (flag byte 0)
        handles = _exchange(bytes([0 if err else 1]) + bytes(handle), self.group)
        handles = [h[1:] if h[0] else None for h in handles]
        if any(h is None for h in handles):
            if self.own:
                ops.peer_free(self.own)
                self.own = None
            raise RuntimeError('peer region allocation failed on rank(s) %s%s' % (
                [r for r, h in enumerate(handles) if h is None], (': ' + err) if err else ''))
        bases = []
        try:
            for r, h in enumerate(handles):
                if r == self.rank:
                    bases.append(self.own)
                    continue
                hb = (C.c_ubyte * 64).from_buffer_copy(h)
                p = C.c_void_p()
                ops.peer_open(hb, C.byref(p))
                bases.append(p.value)
                self._opened.append(p.value)
        except Exception:
            self.close()
            raise
        self._bases = (C.c_void_p * self.world)(*bases)

    def all_reduce(self, t):
        """In-place sum over the ranks of a contiguous fp64 device tensor (n <= cap)."""
        assert t.is_cuda and t.dtype == torch.float64 and t.is_contiguous() and t.numel() <= self.cap
        ops.peer_allreduce_f64(t.data_ptr(), t.numel(), self.cap, self.rank, self.world, self._bases,
                               torch.cuda.current_stream().cuda_stream)

    def timed_out(self, reset=True):
        """0, or 1 + the rank whose slice a wait gave up on (synchronises)."""
        v = C.c_int()
        ops.peer_status(self.own, int(reset), C.byref(v))
        return v.value

    def close(self):
        """Unmap and free (after a barrier: no peer may still write into the own region)."""
        for p in self._opened:
            ops.peer_close(p)
        self._opened = []
        if self.own:
            ops.peer_free(self.own)
            self.own = None


class PeerAllReduce(object):
    """callable(t) -> in-place sum over the ranks; one region per issuing stream.

    A region is built collectively the first time a stream reduces (eager) and
    validated at once: every rank must map every peer's region and one test
    exchange (rank + 1 from each rank) must return the exact sum on every rank
    within the kernel's wait bound.  The verdict is agreed over the process
    group, so if ANY rank fails, ALL ranks switch this reducer to RCCL
    (`fallback`) for the rest of the run -- never a mixed state."""

    def __init__(self, group=None, cap=CAP):
        self.group = group
        self.cap = cap
        self.regions = {}
        self.fallback = None   # the reason, once the ranks agreed to use RCCL instead

    def _agree(self, ok):
        return all(f == b'\x01' for f in _exchange(b'\x01' if ok else b'\x00', self.group))

    def _build(self):
        r, why = None, None
        try:
            r = PeerRegion(self.group, self.cap)
        except Exception as e:   # this rank cannot allocate / map: agreed below
            why = 'region setup: %s' % e
        if self._agree(r is not None):
            world = dist.get_world_size(self.group)
            t = torch.full((8,), float(dist.get_rank(self.group) + 1), dtype=torch.float64,
                           device=torch.cuda.current_device())
            r.all_reduce(t)
            torch.cuda.synchronize()
            good = r.timed_out() == 0 and bool((t == world * (world + 1) / 2.0).all())
            if not good:
                why = 'test exchange returned %s' % t[:2].tolist()
            if self._agree(good):
                return r
        elif why is None:
            why = 'another rank could not set up its region'
        # every rank joins one more exchange before any region is unmapped (no peer may
        # still be writing into it), whether or not it holds a region: a rank that
        # failed in PeerRegion has none, and skipping the round there would leave the
        # others waiting in it.  An exchange, not dist.barrier: on the default group it
        # stays on the lane's own communicator (ProcessGroupNCCL is kept off this path)
        _exchange(b'\x00', self.group)
        if r is not None:
            r.close()
        self.fallback = why or 'a peer rank failed the test exchange'
        import warnings
        warnings.warn('eegan_hip.peer: SyncBN statistics over RCCL instead of the peer-write all-reduce (%s)'
                      % self.fallback)
        return None

    def region(self):
        s = torch.cuda.current_stream()
        r = self.regions.get(s.cuda_stream)
        if r is None and self.fallback is None:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError('eegan_hip.peer: first SyncBN reduction of a stream inside graph capture; run '
                                   'one eager step first (regions are created collectively, outside capture)')
            r = self._build()
            if r is not None:
                self.regions[s.cuda_stream] = r
        return r

    def __call__(self, t):
        if not t.is_cuda:
            fixed_order_sum(t, self.group)   # CPU process groups (gloo tests): the same combine
        elif t.dtype != torch.float64 or not t.is_contiguous() or t.numel() > self.cap:
            dist.all_reduce(t, group=self.group)
        else:
            r = self.region()
            if r is not None:
                r.all_reduce(t)
            elif self.group is None:
                from . import dist as D
                D.all_reduce(t)      # RCCL on the stream's own communicator (capturable)
            else:
                dist.all_reduce(t, group=self.group)

    def timed_out(self):
        return max([r.timed_out() for r in self.regions.values()] or [0])

    def check(self):
        """Raise when a reduction gave up waiting for a peer since the last
        check (its output was poisoned with NaN; the ranks' epochs no longer
        agree, so training cannot continue).  Synchronises the device."""
        t = self.timed_out()
        if t:
            raise RuntimeError('eegan_hip.peer: a SyncBN peer-write all-reduce timed out waiting for rank %d '
                               '(a rank died or stalled > %d s, EEGAN_PEER_WAIT_S); its BN statistics are NaN'
                               % (t - 1, WAIT_S))

    def close(self):
        for r in self.regions.values():
            r.close()
        self.regions = {}


def _exchange(b, group):
    """Every rank's bytes b (equal lengths), in rank order: over the lane's own
    RCCL communicator for the default group (eegan_hip.dist.all_gather_bytes),
    else through the group."""
    if group is None:
        from . import dist as D
        return D.all_gather_bytes(b, torch.cuda.current_device())
    out = [None] * dist.get_world_size(group)
    dist.all_gather_object(out, b, group=group)
    return out


def fixed_order_sum(t, group=None):
    """The peer kernel's combine on a CPU process group: every rank ends with
    0 + m_0 + m_1 + ... + m_{W-1} (fp64, rank order) -- identical bits on all
    ranks, whatever the group's own all-reduce order would be."""
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size(group))]
    dist.all_gather(parts, t.contiguous(), group=group)
    acc = torch.zeros_like(t)
    for p in parts:
        acc += p
    t.copy_(acc)
