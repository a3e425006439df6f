"""Flat-buffer Adam on libeegan_hip.so (replaces torch.optim.Adam of
train.py:252-263).

All parameters of one optimizer are re-homed into ONE contiguous fp32
buffer (parameters become views), their gradients into another, so
zero_grad is one fill and step is one fused kernel launch.  With a process
group, step() first averages the flat gradient buffer across ranks with
bucketed RCCL all-reduces (data parallelism; train.py's DataParallel
gradient reduction).  After each step a generation counter shared by the
parameters is bumped and every conv weight's bf16 packs (forward and
backward-data images, eegan_hip.functional.PackCache) are rebuilt in ONE
batched launch, so no per-layer pack kernel runs in the next forward/backward.

Overlap (world > 1 on the default group): the flat gradient is reduced in
buckets of parameters taken in REVERSE registration order -- the order a
backward completes them -- and a bucket's all-reduce is issued during the
backward, on the stream that wrote its last gradient, as soon as every
parameter in it has received all of its gradient writes.  The kernels write
parameter gradients straight into the flat buffer (functional._grad_sink),
which reports each write here; how many writes a parameter receives in one
zero_grad..step window (1 in a first-order backward, 2 for a conv weight in
the gradient penalty's second-order backward) is learned from the first
window of its kind and then required.  Windows are keyed by the first
parameter written and the backward Function writing it (a first-order
backward and the gradient penalty's double backward write from different
Functions); windows of different kinds can still share a key,
so a key holds every write-count plan learned under it (its first two
windows only learn), and a bucket is
reduced early only when ALL plans still consistent with the writes seen so
far agree it is complete (a plan drops out as soon as a parameter receives
more writes than it allows).  A window that matches no plan raises if it
writes into an already reduced bucket, and its counts are learned at step().
A bucket is reduced early only if all its writes came from the stream that
completes it (the all-reduce is issued there); buckets written from several
streams, or holding a parameter whose gradient arrives any other way
(autograd's own accumulation), are reduced at step(), as are all buckets of
an unlearned window.  EEGAN_GRAD_OVERLAP=0 reduces everything at step().

Communication lane (`comm_stream`, set by the trainer for the optimizers on
the step's critical path): a bucket's all-reduce is issued on that stream
instead -- ordered behind every write issued so far on the writing stream by
an event -- so the rest of the backward on the writing stream does not queue
behind the reduction; step() waits for the lane before averaging and the
Adam launch.  The lane has its own RCCL communicator (eegan_hip.dist.
bind_stream); its reductions keep the plan's bucket order on every rank.
"""
import os

import torch

from ._lib import ops
from .tensor import ptr, stream


def _align(n, a=4):
    return (n + a - 1) // a * a


OVERLAP = os.environ.get('EEGAN_GRAD_OVERLAP', '1') != '0'
# EEGAN_ADAM_PACK=0: Adam over the flat buffer, then the conv weight re-pack as a
# second launch (instead of eegan_adam_pack: one launch, the updated weights packed
# from LDS without reading them back); module constant for A/B
ADAM_PACK = os.environ.get('EEGAN_ADAM_PACK', '1') != '0'


class FlatAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, process_group=None,
                 bucket_bytes=16 << 20):
        params = [p for p in params]
        seen, uniq = set(), []
        for p in params:
            if id(p) not in seen:
                seen.add(id(p))
                uniq.append(p)
        super().__init__(uniq, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.process_group = process_group
        self.params = uniq  # the leaves this optimiser updates (backward(inputs=...))
        dev = uniq[0].device
        offs, n = [], 0
        for p in uniq:
            offs.append(n)
            n += _align(p.numel())
        self.numel = n
        self.flat = torch.zeros(n, dtype=torch.float32, device=dev)
        self.gflat = torch.zeros(n, dtype=torch.float32, device=dev)
        self.m = torch.zeros(n, dtype=torch.float32, device=dev)
        self.v = torch.zeros(n, dtype=torch.float32, device=dev)
        self._gen = [0]
        self._views = []
        with torch.no_grad():
            for p, o in zip(uniq, offs):
                k = p.numel()
                # views keep each parameter's strides (conv weights are channels-last)
                pv = self.flat[o:o + k].as_strided(p.shape, p.stride())
                pv.copy_(p.detach())
                p.data = pv
                g = self.gflat[o:o + k].as_strided(p.shape, p.stride())
                p.grad = g
                p._eegan_gen = self._gen
                p._eegan_opt = self
                self._views.append((p, o, k, g))
        self._pack_sig = None
        self._pack_table = None
        self._pack_total = 0
        self._fused_sig = None
        self._fused_table = None
        self._fused_jobs = 0
        self._fused_total = 0
        self._fused_packs = []
        self.step_count = 0   # host mirror (state_dict); the kernels use step_dev
        self.step_dev = torch.zeros(1, dtype=torch.float64, device=dev)
        self._index = {id(p): i for i, p in enumerate(uniq)}
        self._offs = offs
        self.set_bucket_bytes(bucket_bytes)
        self._plans = {}         # window key -> [(writes per param, early-eligible bucket flags, writing stream per bucket)]
        self._key_seen = {}      # window key -> windows opened under it
        self._late = set()       # params whose gradient went through autograd at least once
        self._win = None
        self.comm_stream = None  # bucket all-reduces on this stream (the trainer's communication lane)
        self.comm_origin = None  # the stream the lane was forked from (the step's origin stream)
        self._comm_used = False

    # ------------------------------------------------------ overlapped DP --
    def set_bucket_bytes(self, nbytes):
        """Reduction buckets: parameter index ranges in reverse registration
        order, >= nbytes each (the last one may be smaller)."""
        self.bucket_elems = max(1, nbytes // 4)
        self.buckets = []       # (lo, hi): params [lo, hi), flat range [offs[lo], end of hi-1)
        hi, acc = len(self.params), 0
        for i in range(len(self.params) - 1, -1, -1):
            acc += _align(self.params[i].numel())
            if acc >= self.bucket_elems or i == 0:
                self.buckets.append((i, hi))
                hi, acc = i, 0
        self._bucket_of = [0] * len(self.params)
        for b, (lo, hi) in enumerate(self.buckets):
            for i in range(lo, hi):
                self._bucket_of[i] = b
        self._plans = {}
        self._key_seen = {}

    def _dp(self):
        import torch.distributed as dist
        from . import dist as D
        if self.process_group is None or not dist.is_initialized():
            return 0
        world = dist.get_world_size(self.process_group)
        if world == 1 and not D.FORCE:
            return 0
        return world

    def _flat_range(self, b):
        lo, hi = self.buckets[b]
        return self._offs[lo], self._offs[hi - 1] + _align(self._views[hi - 1][2])

    def _reduce_bucket(self, b):
        import torch.distributed as dist
        from . import dist as D
        s, e = self._flat_range(b)

        def issue():
            if self.process_group is dist.group.WORLD:
                D.all_reduce(self.gflat[s:e])
            else:
                dist.all_reduce(self.gflat[s:e], group=self.process_group)
        cs = self.comm_stream
        if cs is not None and self.gflat.is_cuda:
            cs.wait_stream(torch.cuda.current_stream())   # behind every gradient write issued so far
            with torch.cuda.stream(cs):
                issue()
            self._comm_used = True
        else:
            issue()
        self._win['done'][b] = True

    def _new_window(self):
        return {'key': None, 'cands': [], 'counts': [0] * len(self.params), 'ready': [],
                'done': [False] * len(self.buckets), 'streams': [None] * len(self.buckets)}

    def flush_ready(self):
        """Reduce the buckets completed by writes that are launched by now
        (called by functional once the writing Function's backward returned)."""
        w = self._win
        if w is None:
            return
        cur = torch.cuda.current_stream().cuda_stream if self.gflat.is_cuda else 0
        for b in w['ready']:
            if w['streams'][b] == cur:   # issued behind every write of the bucket
                self._reduce_bucket(b)
        w['ready'] = []

    def note_grad_write(self, p, site=None):
        """A kernel is about to accumulate into p.grad (functional._grad_sink),
        on the current stream, from backward Function `site`.  True when this
        write completes a bucket (reduced by flush_ready)."""
        w = self._win
        if w is None:
            return False
        i = self._index[id(p)]
        b = self._bucket_of[i]
        if w['key'] is None:
            w['key'] = key = (i, site)
            seen = self._key_seen.get(key, 0)
            self._key_seen[key] = seen + 1
            # a key's plans steer early reductions from its third window on, so
            # two kinds of window sharing a key are both learned first
            w['cands'] = list(self._plans.get(key, ())) if seen >= 2 else []
        w['counts'][i] += 1
        c = w['counts'][i]
        st = torch.cuda.current_stream().cuda_stream if p.is_cuda else 0
        ws = w['streams'][b]
        if ws is None:
            w['streams'][b] = st
        elif ws != st:
            w['streams'][b] = -1     # written from several streams: reduce at step()
        if w['done'][b]:
            raise RuntimeError('FlatAdam: parameter %d received gradient write %d after its bucket was reduced '
                               '(no learned write plan matches this window)' % (i, c))
        # plans that allow fewer writes of p than seen are not this window's
        w['cands'] = [pl for pl in w['cands'] if pl[0][i] >= c]
        if not w['cands'] or w['streams'][b] == -1 or b in w['ready']:
            return False
        lo, hi = self.buckets[b]
        for need, early, _ in w['cands']:
            if not early[b] or any(w['counts'][j] != need[j] for j in range(lo, hi)):
                return False
        w['ready'].append(b)
        return True

    def zero_grad(self, set_to_none=False):
        ops.fill_f32(self.gflat.data_ptr(), self.numel, 0.0, stream())
        for p, o, k, g in self._views:
            if p.grad is None or p.grad.data_ptr() != g.data_ptr():
                p.grad = g
        if OVERLAP and self._dp() and self.process_group is not None:
            import torch.distributed as dist
            if self.process_group is dist.group.WORLD:
                self._win = self._new_window()
                for p in self.params:
                    p._eegan_track = self

    def note_autograd_write(self, p):
        """A kernel Function hands p's gradient to autograd's accumulation
        (no direct write): p's bucket is never reduced early."""
        i = self._index[id(p)]
        self._late.add(i)
        w = self._win
        if w is not None and w['done'][self._bucket_of[i]]:
            raise RuntimeError('FlatAdam: parameter %d accumulated by autograd after its bucket was reduced' % i)

    def _sync_grads(self):
        # gradients that autograd produced out of place (or dropped) are folded back in
        for i, (p, o, k, g) in enumerate(self._views):
            if p.grad is None:
                p.grad = g
                g.zero_()
            elif p.grad.data_ptr() != g.data_ptr():
                g.copy_(p.grad)
                p.grad = g
                self._late.add(i)

    def _allreduce(self):
        world = self._dp()
        if not world:
            return
        w = self._win
        if w is None:   # no overlap: every bucket now
            self._win = w = self._new_window()
        self.flush_ready()
        late_buckets = {self._bucket_of[i] for i in self._late}
        if any(w['done'][b] for b in late_buckets):
            raise RuntimeError('FlatAdam: a bucket with an out-of-place gradient was reduced early')
        for b in range(len(self.buckets)):   # everything not reduced during the backward, in bucket order
            if not w['done'][b]:
                self._reduce_bucket(b)
        if w['key'] is not None:   # learn this window's write counts (a new kind of window under this key)
            need = tuple(w['counts'])
            plans = self._plans.setdefault(w['key'], [])
            if not any(pl[0] == need for pl in plans):
                early = [all(need[j] > 0 and j not in self._late for j in range(lo, hi)) and w['streams'][b] != -1
                         for b, (lo, hi) in enumerate(self.buckets)]
                plans.append((need, early, w['streams'][:]))
        self._win = None
        for p in self.params:
            p._eegan_track = None
        if self._comm_used:
            cur = torch.cuda.current_stream()
            org = self.comm_origin
            if org is None or org.cuda_stream == cur.cuda_stream:
                cur.wait_stream(self.comm_stream)
            else:
                # a lane forked from the origin never waits on the communication lane
                # itself: lane <-> lane waits make the runtime's end-of-capture walk
                # over forked streams recurse without end (stack overflow inside
                # hipStreamEndCapture); the origin joins the lane and this stream
                # waits on the origin, which it was forked from anyway
                org.wait_stream(self.comm_stream)
                cur.wait_stream(org)
            self._comm_used = False
        self.gflat.mul_(1.0 / world)

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        self._sync_grads()
        self._allreduce()
        g = self.param_groups[0]
        b1, b2 = g['betas']
        self.step_count += 1
        if ADAM_PACK and self._fused_plan():
            ops.adam_pack(self.flat.data_ptr(), self.gflat.data_ptr(), self.m.data_ptr(), self.v.data_ptr(), b1, b2,
                          g['lr'], g['eps'], g['weight_decay'], self.step_dev.data_ptr(), self._fused_table.data_ptr(),
                          self._fused_jobs, self._fused_total, stream())
            self._gen[0] += 1
            self._mark_packs(self._fused_packs)
            return loss
        ops.adam(self.flat.data_ptr(), self.gflat.data_ptr(), self.m.data_ptr(), self.v.data_ptr(), self.numel, b1, b2,
                 g['lr'], g['eps'], g['weight_decay'], self.step_dev.data_ptr(), stream())
        self._gen[0] += 1
        self._repack()
        return loss

    def _packed_weights(self):
        """(param, flat offset, cache) of this optimizer's conv weights with bf16 packs."""
        out = []
        for p, o, k, g in self._views:
            c = getattr(p, '_eegan_packcache', None)
            if c is None or p.dim() != 4 or c.scale is not None or (c.fwd is None and c.bwd is None):
                continue
            if not p.is_contiguous(memory_format=torch.channels_last):
                raise RuntimeError('FlatAdam: conv weight %s is not stored channels-last' % (tuple(p.shape),))
            out.append((p, o, c))
        return out

    def _fused_plan(self):
        """The job table of eegan_adam_pack (conv weights as tap tiles, everything
        else -- other parameters and the alignment gaps -- as element ranges),
        rebuilt when the set of packs changes (never inside a capture).  False
        when there is nothing to pack: the plain Adam launch then."""
        ws = self._packed_weights()
        if not ws:
            return False
        sig = tuple((id(c), o, ptr(c.fwd), ptr(c.bwd)) for p, o, c in ws)
        if sig != self._fused_sig:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError('FlatAdam: the set of weight packs changed during graph capture; '
                                   'run an eager warm-up step first')
            rows, pre, pos = [], [0], 0
            for p, o, c in sorted(ws, key=lambda t: t[1]):
                if o > pos:
                    rows += [1, pos, o - pos, 0, 0, 0, 0, 0]
                    pre.append(pre[-1] + ops.adam_range_blocks(o - pos))
                Cout, Cin, R, S = p.shape
                rows += [0, o, ptr(c.fwd), ptr(c.bwd), Cout, Cin, R * S, 0]
                pre.append(pre[-1] + ops.adam_pack_blocks(Cout, Cin, R, S))
                pos = o + p.numel()
            if pos < self.numel:
                rows += [1, pos, self.numel - pos, 0, 0, 0, 0, 0]
                pre.append(pre[-1] + ops.adam_range_blocks(self.numel - pos))
            self._fused_jobs = len(pre) - 1
            self._fused_table = torch.tensor(rows + pre, dtype=torch.int64).to(self.flat.device)
            self._fused_total = pre[-1]
            self._fused_packs = [(p, c) for p, o, c in ws]
            self._fused_sig = sig
        return True

    @staticmethod
    def _mark_packs(packs):
        from .functional import PackCache
        for p, c in packs:
            key = PackCache._key(p)
            if c.fwd is not None:
                c.fwd_key = key
            if c.bwd is not None:
                c.bwd_key = key

    def _repack(self):
        """Refresh the registered bf16 packs of this optimizer's conv weights in
        one launch; their cache keys then match the new generation."""
        from .functional import PackCache
        jobs = []
        for p, o, k, g in self._views:
            c = getattr(p, '_eegan_packcache', None)
            if c is None or p.dim() != 4 or c.scale is not None:
                continue
            if not p.is_contiguous(memory_format=torch.channels_last):
                raise RuntimeError('FlatAdam: conv weight %s is not stored channels-last' % (tuple(p.shape),))
            for tr, buf in ((False, c.fwd), (True, c.bwd)):
                if buf is not None:
                    jobs.append((p, c, tr, buf))
        if not jobs:
            return
        sig = tuple((id(c), tr, buf.data_ptr(), buf.numel()) for p, c, tr, buf in jobs)
        if sig != self._pack_sig:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError('FlatAdam: the set of weight packs changed during graph capture; '
                                   'run an eager warm-up step first')
            rows, pre = [], [0]
            for p, c, tr, buf in jobs:
                Cout, Cin, R, S = p.shape
                rows += [p.data_ptr(), 0, buf.data_ptr(), Cout, Cin, R, S, int(tr)]
                pre.append(pre[-1] + ops.conv_pack_multi_blocks(Cout, Cin, R, S, int(tr)))
            self._pack_table = torch.tensor(rows + pre, dtype=torch.int64).to(self.flat.device)
            self._pack_total = pre[-1]
            self._pack_sig = sig
        ops.conv_pack_weights_multi(self._pack_table.data_ptr(), len(jobs), self._pack_total, stream())
        for p, c, tr, buf in jobs:
            key = PackCache._key(p)
            if tr:
                c.bwd_key = key
            else:
                c.fwd_key = key
