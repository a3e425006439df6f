"""FID leg on the MI355X (reference metrics/FID/inception.py,
fid_score.py:110-228): the HIP InceptionV3 feature network against the oracle
restatement (parity unpinned: torchvision and the pretrained weights are
absent), the fp64 device statistics against np.mean / np.cov and the golden
statistics of the reference's script, and the FID of device statistics against
the reference's value on the same activations."""
import os

import numpy as np
import pytest
import torch

from _util import REPO
from oracle.seeding import seeded_state, seeded_tensor, summary

pytestmark = pytest.mark.gpu
GOLD = os.path.join(REPO, 'tests', 'golden', 'fid.npz')


def test_fid_statistics_match_numpy_and_reference(gpu):
    from metrics.FID.fid_score import MeasureFID
    g = np.load(GOLD)
    for c in ('c0', 'c1'):
        m1, s1 = MeasureFID.device_statistics(torch.from_numpy(g[c + '/act1']).to(gpu))
        m2, s2 = MeasureFID.device_statistics(torch.from_numpy(g[c + '/act2']).to(gpu))
        for got, ref in ((m1, g[c + '/mu1']), (s1, g[c + '/sigma1']), (m2, g[c + '/mu2']), (s2, g[c + '/sigma2'])):
            assert np.abs(got - ref).max() <= 1e-12 * max(1.0, np.abs(ref).max())
        assert np.array_equal(s1, s1.T)   # mirrored tiles: exactly symmetric
        fid = MeasureFID.calculate_frechet_distance(m1, s1, m2, s2)
        assert abs(fid - float(g[c + '/fid'])) <= 1e-9 * abs(float(g[c + '/fid']))
    # pool_3 size: 2048 features, several sample counts, ragged tiles
    rs = np.random.RandomState(1)
    for N, D in ((300, 200), (70, 2048)):
        a = (rs.randn(N, D) * rs.rand(D) + rs.randn(D)).astype(np.float32)
        mu, sig = MeasureFID.device_statistics(torch.from_numpy(a).to(gpu))
        a64 = a.astype(np.float64)
        assert np.abs(mu - a64.mean(0)).max() <= 1e-12 * np.abs(a64).max()
        ref = np.cov(a64, rowvar=False)
        assert np.abs(sig - ref).max() <= 1e-10 * np.abs(ref).max()


def _seeded_inception(gpu, blocks=(3,)):
    from metrics.FID.inception import InceptionV3
    m = InceptionV3(None, list(blocks))
    sd = seeded_state([(k, tuple(v.shape)) for k, v in m.state_dict().items()], 83)
    m.load_state_dict(sd)
    return m.to(gpu), sd


def test_fid_inception_vs_oracle(gpu):
    """Block outputs of the HIP InceptionV3 (all four blocks) vs the oracle's
    fp32 restatement: bf16 activations, so gated like the CNN_ENCODER trunk
    (rel-L2 5e-2)."""
    from oracle import eegan_oracle as O
    from _util import rel_l2
    m, sd = _seeded_inception(gpu, (0, 1, 2, 3))
    x = seeded_tensor('fid:x', (2, 3, 96, 80), 1, 'uniform', 0.0, 1.0)
    outs = m(x.to(gpu))
    refs = O.fid_inception(sd, x, (0, 1, 2, 3))
    assert [tuple(o.shape) for o in outs] == [tuple(r.shape) for r in refs]
    assert tuple(outs[-1].shape) == (2, 2048, 1, 1)
    for k, (o, r) in enumerate(zip(outs, refs)):
        e = rel_l2(o.float().cpu(), r)
        print('PARITY fid/block%d rel_l2=%.3e' % (k, e))
        assert e < 5e-2, (k, e)


def test_fid_end_to_end_device_vs_host_statistics(gpu):
    """FID between two image sets: device statistics vs the reference's host
    path (activations -> float64 numpy -> np.mean / np.cov) on the same
    activations."""
    from metrics.FID.fid_score import MeasureFID
    m, _ = _seeded_inception(gpu)
    g = torch.Generator().manual_seed(4)
    sets = [[torch.rand(8, 3, 64, 64, generator=g) for _ in range(3)],
            [torch.rand(8, 3, 64, 64, generator=g) ** 2 for _ in range(3)]]
    dev = [MeasureFID.activation_statistics(s, m) for s in sets]
    host = []
    for s in sets:
        act = MeasureFID.calculate_activation_statistics(s, m, verbose=False)
        host.append((np.mean(act, axis=0), np.cov(act, rowvar=False)))
    for (md, sd_), (mh, sh) in zip(dev, host):
        assert np.abs(md - mh).max() <= 1e-10 * np.abs(mh).max()
        assert np.abs(sd_ - sh).max() <= 1e-9 * np.abs(sh).max()
    fd = MeasureFID.calculate_frechet_distance(*dev[0], *dev[1])
    fh = MeasureFID.calculate_frechet_distance(*host[0], *host[1])
    assert abs(fd - fh) <= 1e-6 * abs(fh), (fd, fh)
