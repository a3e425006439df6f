"""Shared test helpers (golden loading, fingerprint comparison)."""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
PKG = os.path.join(REPO, 'ee-gan_amd')
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

from oracle.seeding import summary, seeded_state  # noqa: E402


def torchrun_argv(nproc):
    """`python -m torch.distributed.run` for one node with its rendezvous port
    bound atomically: --standalone runs the c10d rendezvous on port 0 and the
    agent's TCPStore binds it itself, so no test picks a port, releases it and
    hands the number to a later bind (round 5's EADDRINUSE race).  The store
    and the workers' MASTER_ADDR stay on 127.0.0.1 (the host name may not
    resolve)."""
    return [sys.executable, '-m', 'torch.distributed.run', '--standalone', '--local-addr', '127.0.0.1',
            '--nnodes=1', '--nproc-per-node', str(nproc)]


_GOLD = None


def golden():
    """Golden vectors captured from the reference (tests/golden/make_golden.py):
    golden.npz (blocks, networks, losses, the round-1 step) and
    golden_steps.npz (the C4 / non-32-width / stage-1 steps)."""
    global _GOLD
    if _GOLD is None:
        _GOLD = {}
        for f in ('golden.npz', 'golden_steps.npz'):
            _GOLD.update(dict(np.load(os.path.join(HERE, 'golden', f))))
    return _GOLD


def spec(name):
    raw = golden()[name + '/spec'].tobytes().decode()
    return [(k, tuple(s)) for k, s in json.loads(raw)]


def golden_state(name, seed):
    return seeded_state(spec(name), seed)


def fp(t):
    """Fingerprint of a tensor in the same format as the golden file."""
    return summary(t)


def assert_close_fp(name, got, ref, rtol, atol):
    """Compare a fingerprint (or a full array) with the reference.  For
    fingerprints the aggregate entries are checked with a tolerance scaled by
    the tensor's abs-sum / sq-sum, the sampled entries element-wise."""
    got = np.asarray(got, np.float64).reshape(-1)
    ref = np.asarray(ref, np.float64).reshape(-1)
    assert got.shape == ref.shape, '%s: shape %s vs %s' % (name, got.shape, ref.shape)
    if ref.size > 4096 or (ref.size >= 6 and ref.size == 6 + 512):
        n = ref[0]
        assert got[0] == n, '%s: numel' % name
        abs_sum, sq = ref[2], ref[3]
        scale = max(abs_sum / n, 1e-30)
        assert abs(got[1] - ref[1]) <= rtol * abs_sum + atol * n, '%s: sum %g vs %g' % (name, got[1], ref[1])
        assert abs(got[2] - ref[2]) <= rtol * abs_sum + atol * n, '%s: abs-sum %g vs %g' % (name, got[2], ref[2])
        assert abs(got[3] - ref[3]) <= 2 * rtol * sq + atol * n * scale, '%s: sq-sum %g vs %g' % (name, got[3], ref[3])
        a, b = got[6:], ref[6:]
    else:
        a, b = got, ref
    err = np.abs(a - b)
    tol = atol + rtol * np.abs(b)
    bad = np.nonzero(err > tol)[0]
    assert bad.size == 0, '%s: %d/%d mismatches, max err %.3g (first idx %d: %r vs %r)' % (
        name, bad.size, a.size, err.max(), bad[0], a[bad[0]], b[bad[0]])


def rel_l2(a, b):
    a = a.detach().double().reshape(-1).cpu()
    b = b.detach().double().reshape(-1).cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def conv_knob(monkeypatch, key, value):
    """Set one conv planner / kernel-path knob inside EEGAN_CONV ("key=value,...",
    read per launch by csrc/conv.hip's knob()); monkeypatch restores the variable."""
    cur = os.environ.get('EEGAN_CONV', '')
    items = [kv for kv in cur.split(',') if kv and kv.split('=')[0] != key]
    items.append('%s=%s' % (key, value))
    monkeypatch.setenv('EEGAN_CONV', ','.join(items))
