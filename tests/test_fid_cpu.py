"""FID leg on the CPU: the host Frechet distance against the
golden values produced by the reference's own MeasureFID.calculate_frechet_distance
(tests/golden/make_fid_golden.py), incl. the singular-product fallback, and its
known answers."""
import os

import numpy as np

from _util import REPO

GOLD = os.path.join(REPO, 'tests', 'golden', 'fid.npz')


def test_frechet_distance_matches_reference():
    from metrics.FID.fid_score import MeasureFID
    g = np.load(GOLD)
    for c in ('c0', 'c1', 'sing'):
        got = MeasureFID.calculate_frechet_distance(g[c + '/mu1'], g[c + '/sigma1'], g[c + '/mu2'], g[c + '/sigma2'])
        ref = float(g[c + '/fid'])
        assert abs(got - ref) <= 1e-9 * max(1.0, abs(ref)), (c, got, ref)


def test_frechet_distance_known_answers():
    from metrics.FID.fid_score import MeasureFID
    rs = np.random.RandomState(0)
    a = rs.randn(200, 8)
    mu, sig = a.mean(0), np.cov(a, rowvar=False)
    assert abs(MeasureFID.calculate_frechet_distance(mu, sig, mu, sig)) < 1e-8
    d = rs.randn(8)
    assert abs(MeasureFID.calculate_frechet_distance(mu, sig, mu + d, sig) - d.dot(d)) < 1e-8
