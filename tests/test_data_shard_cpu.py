"""The data side of an unchanged train.py at N > 1, on the CPU.

The reference's DataParallel scatters one batch over its GPUs
(train.py:220-228).  One process per GPU instead runs train.py once per rank,
seeded alike (train.py:521-525), so the drop-in dataset shards itself over the
ranks and moves ranks > 0 onto their own random streams (datasets.TextDataset,
eegan_hip.launch.offset_rank_rngs); the models broadcast rank 0's weights at
the first forward (eegan_hip.dist.broadcast_state).  Checked here: the shard
arithmetic, train.py's default-collated DataLoader over HostImages (draws in
torchvision's order from the global generator, picklable for workers), the
stream offsets, and -- in a two-rank torchrun job over gloo shaped like
train.py -- disjoint images, different noise, an epoch that covers the split
once, and identical weights after the broadcast."""
import os
import pickle
import subprocess
import sys

import numpy as np
import pytest
import torch

from _util import torchrun_argv  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import _pipeline_data as PD  # noqa: E402



@pytest.mark.parametrize('world', [1, 2, 3, 4])
def test_shard_indices(tmp_path, world):
    import datasets as DS
    PD.build(str(tmp_path))
    n = len(PD.SIZES)
    seen = []
    for r in range(world):
        ds = DS.TextDataset(str(tmp_path), 'bird', shard=(r, world)) if world > 1 else \
            DS.TextDataset(str(tmp_path), 'bird', shard=(0, 1))
        assert len(ds) == n // world
        idx = [ds.base_index(i) for i in range(len(ds))]
        assert idx == list(range(r, (n // world) * world, world))
        for i in range(len(ds)):
            key = ds[i][0][4]
            assert key == ds.filenames[idx[i]]
        with pytest.raises(IndexError):
            ds.base_index(len(ds))
        seen += idx
    assert sorted(seen) == list(range((n // world) * world))
    with pytest.raises(ValueError):
        DS.TextDataset(str(tmp_path), 'bird', shard=(2, 2))


def test_default_collate_host_images(tmp_path):
    """train.py's DataLoader (default collate) over the drop-in dataset: `imgs`
    is one lazy entry per scale; the crop/flip draws are the ones torchvision's
    transform takes per sample from the global generator."""
    import datasets as DS
    from eegan_hip.pipeline import bbox_crop_box, resized_size, draw_crop_flip
    PD.build(str(tmp_path))
    ds = DS.TextDataset(str(tmp_path), 'bird', shard=(0, 1))
    torch.manual_seed(11)
    dl = torch.utils.data.DataLoader(ds, batch_size=3, drop_last=True, shuffle=False, num_workers=0)
    it = iter(dl)                       # draws the loader's base seed
    g = torch.Generator()
    g.set_state(torch.get_rng_state())
    basic, attrs, unpair = next(it)
    imgs, caps, cap_lens, cls_ids, keys = basic
    assert isinstance(imgs, DS.HostImageBatch) and len(imgs) == 3
    assert [tuple(im.shape) for im in imgs] == [(3, 3, 64, 64), (3, 3, 128, 128), (3, 3, 256, 256)]
    assert tuple(caps.shape) == (3, 20, 1) and list(keys) == ['img0', 'img1', 'img2']
    for k, (arr, bbox) in enumerate(imgs.records):
        x1, y1, x2, y2 = bbox_crop_box(arr.shape[1], arr.shape[0], bbox)
        nw, nh = resized_size(x2 - x1, y2 - y1, 304)
        assert imgs.draws[k] == draw_crop_flip(nh, nw, 256, g)
        w, h = PD.SIZES[k]
        assert np.array_equal(arr, PD.image(k, w, h))
    # the global generator advanced exactly as torchvision's draws would advance it
    assert torch.equal(torch.rand(4), torch.rand(4, generator=g))
    back = pickle.loads(pickle.dumps(imgs))      # a DataLoader worker returns it by pickle
    assert back.draws == imgs.draws and len(back) == 3 and back._outs is None
    with pytest.raises(IndexError):
        imgs[3]


def test_offset_rank_rngs(monkeypatch):
    import random
    from eegan_hip import launch

    def draws(rank):
        monkeypatch.setattr(launch, '_STATE', {'pinned': None, 'pg': False, 'rng_offset': None})
        random.seed(3407)
        np.random.seed(3407)
        torch.manual_seed(3407)
        launch.offset_rank_rngs(rank)
        launch.offset_rank_rngs(rank)    # once per process
        return torch.randn(5), np.random.randint(0, 1 << 30, 5), random.random()

    s = torch.initial_seed()
    try:
        r0, r1, r1b, r2 = draws(0), draws(1), draws(1), draws(2)
    finally:
        torch.manual_seed(s)
    torch.manual_seed(3407)
    np.random.seed(3407)
    assert torch.equal(r0[0], torch.randn(5)) and np.array_equal(r0[1], np.random.randint(0, 1 << 30, 5))
    assert torch.equal(r1[0], r1b[0]) and np.array_equal(r1[1], r1b[1]) and r1[2] == r1b[2]
    for a, b in ((r0, r1), (r0, r2), (r1, r2)):
        assert not torch.equal(a[0], b[0]) and not np.array_equal(a[1], b[1]) and a[2] != b[2]


def test_mp_child_skips_launch(monkeypatch):
    """A DataLoader worker (a multiprocessing child with the rank's env) must
    not pin or join: train.py's spawned workers re-import its modules."""
    import multiprocessing
    from eegan_hip import launch
    monkeypatch.setenv('LOCAL_RANK', '1')
    monkeypatch.setenv('LOCAL_WORLD_SIZE', '2')
    monkeypatch.setenv('WORLD_SIZE', '2')
    monkeypatch.delenv('EEGAN_AUTO_DIST', raising=False)
    monkeypatch.setattr(launch, '_STATE', {'pinned': None, 'pg': False, 'rng_offset': None})
    called = []
    monkeypatch.setattr(launch, 'pin_rank_device', lambda: called.append('pin'))
    monkeypatch.setattr(launch, 'init_process_group', lambda: called.append('pg'))
    launch.setup()
    assert called == ['pin', 'pg']                  # the rank process itself
    called.clear()
    # a 'spawn' child still importing the parent's main module (parent_process() not set yet)
    monkeypatch.setattr(sys, 'argv', ['-c', '--multiprocessing-fork'])
    launch.setup()
    monkeypatch.setattr(sys, 'argv', ['x'])
    monkeypatch.setattr(multiprocessing.current_process(), '_inheriting', True, raising=False)
    launch.setup()
    monkeypatch.setattr(multiprocessing.current_process(), '_inheriting', False, raising=False)
    monkeypatch.setattr(multiprocessing, 'parent_process', lambda: object())   # a bootstrapped child
    launch.setup()
    assert called == []


def test_pin_after_runtime_start_selects_device(monkeypatch):
    """The runtime already up: the rank's device is selected with set_device."""
    from eegan_hip import launch
    monkeypatch.setenv('LOCAL_RANK', '3')
    monkeypatch.setenv('LOCAL_WORLD_SIZE', '4')
    monkeypatch.setenv('WORLD_SIZE', '4')
    monkeypatch.delenv('EEGAN_AUTO_DIST', raising=False)
    monkeypatch.setattr(launch, '_STATE', {'pinned': None, 'pg': False, 'rng_offset': None})
    monkeypatch.setattr(torch.cuda, 'is_initialized', lambda: True)
    monkeypatch.setattr(torch.cuda, 'device_count', lambda: 2)
    sel = []
    monkeypatch.setattr(torch.cuda, 'set_device', lambda i: sel.append(i))
    assert launch.pin_rank_device() == 'set_device:1' and sel == [1]
    monkeypatch.setattr(launch, '_STATE', {'pinned': None, 'pg': False, 'rng_offset': None})
    monkeypatch.setattr(torch.cuda, 'device_count', lambda: 0)
    with pytest.raises(RuntimeError, match='no visible GPU'):
        launch.pin_rank_device()


def test_uuid_devices_counted_without_runtime(monkeypatch):
    from eegan_hip import launch
    for k in ('ROCR_VISIBLE_DEVICES', 'HIP_VISIBLE_DEVICES', 'CUDA_VISIBLE_DEVICES'):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv('ROCR_VISIBLE_DEVICES', 'GPU-aa,GPU-bb,GPU-cc')
    monkeypatch.setattr(torch.cuda, 'device_count', lambda: (_ for _ in ()).throw(AssertionError('runtime')))
    assert launch._device_count() == 3
    monkeypatch.setenv('LOCAL_RANK', '1')
    monkeypatch.setenv('LOCAL_WORLD_SIZE', '3')
    monkeypatch.setenv('WORLD_SIZE', '3')
    monkeypatch.delenv('EEGAN_AUTO_DIST', raising=False)
    monkeypatch.setattr(launch, '_STATE', {'pinned': None, 'pg': False, 'rng_offset': None})
    monkeypatch.setattr(torch.cuda, 'is_initialized', lambda: False)
    assert launch.pin_rank_device() == 'GPU-bb'
    assert os.environ['ROCR_VISIBLE_DEVICES'] == 'GPU-bb' and os.environ['HIP_VISIBLE_DEVICES'] == '0'


def test_torchrun_ranks_draw_their_own_data(tmp_path):
    """Two ranks of a train.py-shaped job (gloo, CPU): seeded alike, each
    builds TextDataset + DataLoader(shuffle=True) and draws noise as train.py
    does; nothing in the script mentions ranks."""
    data = tmp_path / 'data'
    PD.build(str(data))
    cmd = torchrun_argv(2) + [os.path.join(HERE, 'shard_worker.py'), str(data), str(tmp_path)]
    env = dict(os.environ, OMP_NUM_THREADS='1', EEGAN_DIST_BACKEND='gloo')
    env.pop('EEGAN_AUTO_DIST', None)
    r = subprocess.run(cmd, env=env, timeout=240, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = [torch.load(os.path.join(tmp_path, 'shard_rank%d.pt' % i)) for i in range(2)]
    for rank, x in enumerate(res):
        assert x['len'] == len(PD.SIZES) // 2
        assert all(int(k[3:]) % 2 == rank for ep in x['epochs'] for k in ep)
    for e in range(2):   # per epoch: disjoint, and together the whole split once
        k0, k1 = res[0]['epochs'][e], res[1]['epochs'][e]
        assert not set(k0) & set(k1)
        assert sorted(k0 + k1) == sorted('img%d' % i for i in range(len(PD.SIZES)))
    assert not torch.equal(res[0]['noise'], res[1]['noise'])
    assert res[0]['draws'] != res[1]['draws'] or res[0]['epochs'] != res[1]['epochs']
    assert not torch.equal(res[0]['init'], res[1]['init'])        # built from the offset streams
    assert torch.equal(res[0]['after'], res[1]['after'])          # rank 0's weights after the broadcast
    assert torch.equal(res[0]['after'], res[0]['init'])
