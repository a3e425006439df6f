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
"""
import torch

from ._lib import ops
from .tensor import stream


def _align(n, a=4):
    return (n + a - 1) // a * a


class FlatAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, process_group=None,
                 bucket_bytes=64 << 20):
        params = [p for p in params]
        seen, uniq = set(), []
        for p in params:
            if id(p) not in seen:
                seen.add(id(p))
                uniq.append(p)
        super().__init__(uniq, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.process_group = process_group
        self.params = uniq  # the leaves this optimiser updates (backward(inputs=...))
        self.bucket_elems = max(1, bucket_bytes // 4)
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
                self._views.append((p, o, k, g))
        self._pack_sig = None
        self._pack_table = None
        self._pack_total = 0
        self.step_count = 0   # host mirror (state_dict); the kernels use step_dev
        self.step_dev = torch.zeros(1, dtype=torch.float64, device=dev)

    def zero_grad(self, set_to_none=False):
        ops.fill_f32(self.gflat.data_ptr(), self.numel, 0.0, stream())
        for p, o, k, g in self._views:
            if p.grad is None or p.grad.data_ptr() != g.data_ptr():
                p.grad = g

    def _sync_grads(self):
        # gradients that autograd produced out of place (or dropped) are folded back in
        for p, o, k, g in self._views:
            if p.grad is None:
                p.grad = g
                g.zero_()
            elif p.grad.data_ptr() != g.data_ptr():
                g.copy_(p.grad)
                p.grad = g

    def _allreduce(self):
        import torch.distributed as dist
        from . import dist as D
        if self.process_group is None or not dist.is_initialized() or (
                dist.get_world_size(self.process_group) == 1 and not D.FORCE):
            return
        world = dist.get_world_size(self.process_group)
        world_pg = self.process_group is dist.group.WORLD
        for s in range(0, self.numel, self.bucket_elems):
            if world_pg:
                D.all_reduce(self.gflat[s:s + self.bucket_elems])
            else:
                dist.all_reduce(self.gflat[s:s + self.bucket_elems], group=self.process_group)
        self.gflat.mul_(1.0 / world)

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        self._sync_grads()
        self._allreduce()
        g = self.param_groups[0]
        b1, b2 = g['betas']
        self.step_count += 1
        ops.adam(self.flat.data_ptr(), self.gflat.data_ptr(), self.m.data_ptr(), self.v.data_ptr(), self.numel, b1, b2,
                 g['lr'], g['eps'], g['weight_decay'], self.step_dev.data_ptr(), stream())
        self._gen[0] += 1
        self._repack()
        return loss

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
