"""The drop-in boundary at N > 1 on one GPU box: two ranks (torchrun, gloo --
RCCL refuses two ranks on one device) run the reference train.py's data side and inner
step (tests/dp_dropin_worker.py: TextDataset + DataLoader(shuffle=True) after
train.py's seeding, torch.optim.Adam, nn.DataParallel-wrapped D and
ATTR_Enhance, words_loss / sent_loss from miscc.DAMSM_losses, no rank and no
synchronisation call anywhere).  Checked: each rank draws its own images and
noise; the ranks end the
step with bit-identical parameters (gradient averaging by the models' own
post-accumulate-grad hooks), and they match ONE process stepping the whole
batch (the reference's DataParallel semantics: global-batch SyncBN
statistics with the multi-device numerics, global DAMSM similarity matrices,
means over the global batch) within bf16 rounding."""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

from _util import torchrun_argv  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))



def test_dropin_train_step_two_ranks(gpu, tmp_path, monkeypatch):
    """Two ranks of train.py's data + inner step (tests/dp_dropin_worker.py:
    no rank, no slicing, no synchronisation call anywhere in it).  Each rank
    must draw its OWN images (disjoint stride-2 shards of the split), noise
    and initial weights from its own random streams, start from rank 0's
    weights (broadcast at the first forward), end bit-identical to the other
    rank, and match ONE process stepping the union of the two batches."""
    sys.path.insert(0, HERE)
    import _pipeline_data as PD
    data = tmp_path / 'data'
    PD.build(str(data))
    cmd = torchrun_argv(2) + [os.path.join(HERE, 'dp_dropin_worker.py'), str(data), str(tmp_path)]
    # the worker never calls torch.distributed / eegan_hip.dist: importing the drop-in
    # modules under torchrun pins each rank's GPU and starts the group (eegan_hip.launch);
    # gloo because both ranks share this box's one GPU (RCCL refuses that)
    env = dict(os.environ, OMP_NUM_THREADS='2', EEGAN_DIST_BACKEND='gloo')
    env.pop('EEGAN_AUTO_DIST', None)
    r = subprocess.run(cmd, env=env, timeout=240, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    ranks = [torch.load(os.path.join(tmp_path, 'rank%d.pt' % i)) for i in range(2)]
    for i, rk in enumerate(ranks):   # train.py:513's CUDA_VISIBLE_DEVICES=1 did not unpin the rank's device
        print('DP2 rank', i, 'device pin', rk['info'], 'keys', rk['batch']['keys'])
        assert rk['info']['device_count'] == 1 and rk['info']['hip'] == '0', rk['info']
        assert rk['info']['len'] == len(PD.SIZES) // 2
        assert rk['info']['base'] == list(range(i, len(PD.SIZES), 2))   # the rank's stride-2 shard
        assert all(int(k[3:]) % 2 == i for k in rk['batch']['keys'])
    b0, b1 = ranks[0]['batch'], ranks[1]['batch']
    assert not set(b0['keys']) & set(b1['keys'])                       # disjoint images
    assert not torch.equal(b0['noise'], b1['noise'])                   # train.py:189 differs per rank
    g0, g1 = ranks[0]['init']['g'], ranks[1]['init']['g']
    assert any(not torch.equal(g0[k], g1[k]) for k in g0)              # built from the offset streams
    p0, p1 = ranks[0]['params'], ranks[1]['params']
    assert set(p0) == set(p1)
    for k in p0:   # rank 0's weights broadcast, averaged gradients -> identical Adam steps
        assert torch.equal(p0[k], p1[k]), k
    # DAMSM losses are global: the same value on both ranks
    for k in ('s', 'w', 'a'):
        assert ranks[0]['rec'][k] == ranks[1]['rec'][k], k

    import dp_dropin_worker as W
    from eegan_hip import functional as Fn
    monkeypatch.setattr(Fn, 'SYNC_BN_FORCE_MULTI', True)   # the reference's multi-device BN numerics
    rec, params = W.replay(ranks, gpu, ranks[0]['info']['n_words'])
    for k, v in rec.items():
        got = 0.5 * (ranks[0]['rec'][k] + ranks[1]['rec'][k])   # per-rank means over equal halves
        e = abs(got - v) / max(abs(v), 1e-3)
        print('DP2 %-4s 2-rank %.6g  1-process %.6g  rel %.2e' % (k, got, v, e))
        assert e < (0.08 if k.startswith('gp') else 3e-2), (k, got, v)
    worst = 0.0
    for k, v in params.items():
        a, b = p0[k].double().reshape(-1), v.double().reshape(-1)
        e = float((a - b).norm() / b.norm().clamp_min(1e-30))
        worst = max(worst, e)
        assert e < 2e-2, (k, e)
    print('DP2 worst post-step parameter rel-L2 vs one process: %.3e' % worst)


def test_flat_adam_overlapped_allreduce_two_ranks(gpu, tmp_path):
    """The trainer path (FlatAdam) at N = 2 on one GPU (gloo): gradient
    buckets all-reduced during the backward (EEGAN_GRAD_OVERLAP=1, default)
    give parameters bit-identical to reducing everything at step() (=0), the
    two ranks agree, and the overlap actually happened (buckets reduced from
    inside the backward for every optimizer of the third step).  The default
    step runs the largest D's and the generator's reductions on communication
    lanes (trainer.COMM_LANES) and the generator's stage 2-3 branches on a
    second stream (trainer.GEN_SIDE); both off ('plain') gives the same bits."""
    res = {}
    for tag, ov, extra in (('ov', '1', {}), ('seq', '0', {}),
                           ('plain', '1', {'DP_GEN_SIDE': '0', 'DP_COMM_LANES': '0'})):
        cmd = torchrun_argv(2) + [os.path.join(HERE, 'dp_trainer_worker.py'), str(tmp_path), tag]
        env = dict(os.environ, OMP_NUM_THREADS='2', EEGAN_GRAD_OVERLAP=ov, **extra)
        r = subprocess.run(cmd, env=env, timeout=240, capture_output=True, text=True)
        assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
        res[tag] = [torch.load(os.path.join(tmp_path, 'rank%d_%s.pt' % (i, tag))) for i in range(2)]
    for tag in res:
        for a, b in zip(res[tag][0]['params'], res[tag][1]['params']):
            assert torch.equal(a, b), tag
    for tag in ('seq', 'plain'):
        for a, b in zip(res['ov'][0]['params'], res[tag][0]['params']):
            assert torch.equal(a, b), tag
    print('overlap: buckets reduced inside backward per optimizer', res['ov'][0]['early'],
          'of', res['ov'][0]['buckets'], 'comm lanes', res['ov'][0]['comm_lanes'])
    assert all(e > 0 for e in res['ov'][0]['early']), res['ov'][0]['early']
    assert all(e == 0 for e in res['seq'][0]['early'])
    assert res['ov'][0]['comm_lanes'] == [True, False, False, True]      # optimizerG, D64, D128, D256
    assert not any(res['plain'][0]['comm_lanes'])


def test_force_dist_captured_step_with_comm_lanes(gpu, tmp_path):
    """EEGAN_FORCE_DIST=1 (one rank, RCCL): the data-parallel step with every
    collective issued on its lane's own communicator -- the gradient buckets of
    the largest D and of the generator on their communication lanes
    (trainer.COMM_LANES) -- captures and replays bit-identical to the eager
    step and to the step with the buckets reduced in their writing lanes."""
    res = {}
    for tag, mode, lanes in (('eager', 'eager', '1'), ('graph', 'graph', '1'), ('inlane', 'graph', '0')):
        cmd = torchrun_argv(1) + [os.path.join(HERE, 'dp_force_worker.py'), str(tmp_path), tag, mode]
        env = dict(os.environ, OMP_NUM_THREADS='2', EEGAN_FORCE_DIST='1', DP_COMM_LANES=lanes)
        env.pop('EEGAN_DIST_BACKEND', None)
        r = subprocess.run(cmd, env=env, timeout=240, capture_output=True, text=True)
        assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
        res[tag] = torch.load(os.path.join(tmp_path, 'force_%s.pt' % tag))
    assert res['graph']['comm_lanes'] == [True, False, False, True]
    assert not any(res['inlane']['comm_lanes'])
    d = (res['graph']['state'] - res['eager']['state']).abs().max()
    print('FORCE_DIST max |graph - eager| %.3e' % float(d))
    assert torch.equal(res['graph']['state'], res['eager']['state'])
    assert torch.equal(res['graph']['state'], res['inlane']['state'])


def test_bench_gpus_2_launches_two_ranks(gpu):
    """`python bench.py --gpus 2` with no launcher (the driver's N = 1 command
    form with N = 2) starts a two-rank child job and relays rank 0's line for
    2 GPUs and the global batch of both ranks.  Both ranks share this box's
    one GPU (EEGAN_SHARE_GPU=1, gloo: RCCL refuses two ranks on one device),
    so the number itself is a rehearsal, not a 2-GPU measurement."""
    env = dict(os.environ, EEGAN_SHARE_GPU='1', EEGAN_DIST_BACKEND='gloo', OMP_NUM_THREADS='2')
    env.pop('WORLD_SIZE', None)
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(HERE), 'bench.py'), '--gpus', '2',
                        '--steps', '2', '--warmup', '1', '--no-cpu-baseline', '--timing-steps', '1'],
                       env=env, timeout=400, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    print('bench --gpus 2 (two ranks on one GPU):', rec['value'], rec['unit'], rec['execution'])
    assert rec['n_gpus'] == 2 and rec['config']['global_batch'] == 32 and rec['config']['parallelism'] == 'dp2'
    assert rec['value'] > 0 and rec['steps'] == 2
