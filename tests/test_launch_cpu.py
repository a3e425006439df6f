"""eegan_hip.launch on the CPU: the rank -> GPU pin arithmetic over the
visible-device environment, and an unchanged-train.py-shaped torchrun job
whose ranks are joined by importing the drop-in modules alone (gloo), or,
with the auto start switched off, refuse to train unsynchronised."""
import os
import subprocess
import sys

import pytest
import torch

from _util import torchrun_argv  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))



@pytest.mark.parametrize('env,n,want', [
    ({}, 8, ['0', '1', '2', '3', '4', '5', '6', '7']),
    ({'CUDA_VISIBLE_DEVICES': '4,5,6,7'}, 4, ['4', '5', '6', '7']),
    ({'HIP_VISIBLE_DEVICES': '2,3', 'CUDA_VISIBLE_DEVICES': '0'}, 2, ['2', '3']),   # HIP_ wins, as in the runtime
    ({'ROCR_VISIBLE_DEVICES': '3,5'}, 2, ['3', '5']),
    ({'ROCR_VISIBLE_DEVICES': '3,5,6', 'HIP_VISIBLE_DEVICES': '2,0'}, 2, ['6', '3']),
    ({'ROCR_VISIBLE_DEVICES': 'GPU-aa,GPU-bb', 'CUDA_VISIBLE_DEVICES': '1,7'}, 1, ['GPU-bb']),   # stops at 7
])
def test_visible_physical(monkeypatch, env, n, want):
    from eegan_hip import launch
    for k in ('ROCR_VISIBLE_DEVICES', 'HIP_VISIBLE_DEVICES', 'CUDA_VISIBLE_DEVICES'):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    assert launch._visible_physical(n) == want


def test_pin_sets_rank_device(monkeypatch):
    from eegan_hip import launch
    for k in ('ROCR_VISIBLE_DEVICES', 'HIP_VISIBLE_DEVICES'):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv('CUDA_VISIBLE_DEVICES', '4,5,6,7')
    monkeypatch.setenv('LOCAL_RANK', '2')
    monkeypatch.setenv('LOCAL_WORLD_SIZE', '4')
    monkeypatch.setenv('WORLD_SIZE', '4')
    monkeypatch.delenv('EEGAN_AUTO_DIST', raising=False)
    monkeypatch.setattr(launch, '_STATE', {'pinned': None, 'pg': False})
    monkeypatch.setattr(torch.cuda, 'device_count', lambda: 4)
    monkeypatch.setattr(torch.cuda, 'is_initialized', lambda: False)
    assert launch.pin_rank_device() == '6'
    assert os.environ['ROCR_VISIBLE_DEVICES'] == '6' and os.environ['HIP_VISIBLE_DEVICES'] == '0'
    assert 'CUDA_VISIBLE_DEVICES' not in os.environ
    # EEGAN_AUTO_DIST=0 and non-torchrun processes are left alone
    monkeypatch.setattr(launch, '_STATE', {'pinned': None, 'pg': False})
    monkeypatch.setenv('EEGAN_AUTO_DIST', '0')
    assert launch.pin_rank_device() is None
    monkeypatch.delenv('EEGAN_AUTO_DIST')
    monkeypatch.delenv('LOCAL_WORLD_SIZE')
    assert launch.pin_rank_device() is None


@pytest.mark.parametrize('auto', ['1', '0'])
def test_torchrun_ranks_join_at_import(tmp_path, auto):
    cmd = torchrun_argv(2) + [os.path.join(HERE, 'launch_worker.py'), str(tmp_path)]
    env = dict(os.environ, OMP_NUM_THREADS='1', EEGAN_AUTO_DIST=auto, EEGAN_DIST_BACKEND='gloo')
    r = subprocess.run(cmd, env=env, timeout=180, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = [torch.load(os.path.join(tmp_path, 'launch_rank%d.pt' % i)) for i in range(2)]
    if auto == '1':
        assert all(x['initialized'] and x['world'] == 2 and x['sum'] == 3.0 for x in res), res
        assert sorted(x['rank'] for x in res) == [0, 1]
    else:
        assert all(not x['initialized'] and x['raised'] for x in res), res


def test_peer_timeout_raises_on_trainer_path(monkeypatch):
    """A SyncBN peer-write reduction that gave up waiting for a peer (its
    output poisoned with NaN, csrc/peer.hip) must stop training: the trainer's
    periodic check and its state_dict raise."""
    from eegan_hip import functional as Fn
    from eegan_hip.peer import PeerAllReduce
    from eegan_hip.trainer import Trainer
    red = PeerAllReduce.__new__(PeerAllReduce)
    red.regions = {}
    monkeypatch.setattr(PeerAllReduce, 'timed_out', lambda self: 0)
    monkeypatch.setattr(Fn, 'SYNC_BN_ALLREDUCE', red)
    Trainer.check_collectives()   # healthy: no error
    monkeypatch.setattr(PeerAllReduce, 'timed_out', lambda self: 1 + 3)   # gave up on rank 3
    with pytest.raises(RuntimeError, match='timed out waiting for rank 3'):
        Trainer.check_collectives()
    T = Trainer.__new__(Trainer)
    with pytest.raises(RuntimeError, match='timed out'):
        T.state_dict()


def test_peer_timeout_blocks_dropin_checkpoint(monkeypatch):
    """Under an unchanged train.py (its own loop, train.py:310-318 saving
    netG / attr_enhance / netsD state_dicts directly), a timed-out SyncBN peer
    reduction must stop the checkpoint: every drop-in model's state_dict --
    also through DataParallelWithCallback / nn.DataParallel -- checks first."""
    import torch.nn as nn
    import models
    from sync_batchnorm import DataParallelWithCallback
    from eegan_hip import functional as Fn
    from eegan_hip.peer import PeerAllReduce
    red = PeerAllReduce.__new__(PeerAllReduce)
    red.regions = {}
    monkeypatch.setattr(Fn, 'SYNC_BN_ALLREDUCE', red)
    monkeypatch.setattr(PeerAllReduce, 'timed_out', lambda self: 0)
    nets = [DataParallelWithCallback(models.Gen(8, 100)), nn.DataParallel(models.ATTR_Enhance()),
            nn.DataParallel(models.Dis64(8)), models.Dis256(8, True, 200)]
    for n in nets:
        n.state_dict()    # healthy: no error
    monkeypatch.setattr(PeerAllReduce, 'timed_out', lambda self: 1 + 1)
    for n in nets:
        with pytest.raises(RuntimeError, match='timed out waiting for rank 1'):
            n.state_dict()
