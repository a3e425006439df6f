"""SyncBN peer-write all-reduce (EEGAN_SYNCBN_PEER=1; eegan_hip.peer,
csrc/peer.hip) on the GPU: two torchrun ranks share one MI355X (IPC-mapped
regions, gloo for the handle exchange; RCCL refuses two ranks on one device).
Checked: every reduced message -- eager and from replays of a captured graph --
equals the fixed-order fp64 sum 0 + m_0 + m_1 bit for bit on both ranks, no
wait timed out, SyncBN forward / input gradient / running_var are identical
with the peer path and the group's all-reduce, and the trainer path's three
steps (tests/dp_trainer_worker.py) end with the same parameters as with the
default reduction.  Reference: the statistics exchange of
sync_batchnorm/batchnorm.py:90-111."""
import os
import subprocess
import sys

import pytest
import torch


pytestmark = pytest.mark.gpu
from _util import torchrun_argv  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def _torchrun(script, *args, env=None):
    cmd = torchrun_argv(2) + [os.path.join(HERE, script)] + list(args)
    r = subprocess.run(cmd, env=dict(os.environ, OMP_NUM_THREADS='2', **(env or {})), timeout=240,
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]


def test_peer_allreduce_two_ranks(gpu, tmp_path):
    _torchrun('peer_worker.py', str(tmp_path))
    ranks = [torch.load(os.path.join(tmp_path, 'peer%d.pt' % r)) for r in range(2)]
    for res in ranks:
        assert res['timed_out'] == 0
        for got, want in res['eager']:
            assert torch.equal(got, want)
        for rep in res['graph']:
            for got, want in rep:
                assert torch.equal(got, want)
        for a, b in zip(res['bn']['peer'], res['bn']['group']):
            assert torch.equal(a, b)
    print('PEER one-shot all-reduce, 8 KB fp64, 2 ranks on one GPU: %.2f us per call'
          % max(r['us_per_call'] for r in ranks))


def test_trainer_steps_with_peer_syncbn(gpu, tmp_path):
    res = {}
    for tag, peer in (('peer', '1'), ('group', '0')):
        _torchrun('dp_trainer_worker.py', str(tmp_path), tag, env={'EEGAN_SYNCBN_PEER': peer})
        res[tag] = [torch.load(os.path.join(tmp_path, 'rank%d_%s.pt' % (i, tag))) for i in range(2)]
    for a, b in zip(res['peer'][0]['params'], res['peer'][1]['params']):
        assert torch.equal(a, b)
    for a, b in zip(res['peer'][0]['params'], res['group'][0]['params']):
        assert torch.equal(a, b)
