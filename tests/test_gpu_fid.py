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


def _text_only_dataset(root, n_img=8, cpi=10, words=60, seed=5):
    """The test split of a TextOnlyDataset in the reference's layout (captions.pickle,
    attributes/EE-GAN.pickle, test/filenames.pickle, test/class_info.pickle)."""
    import pickle
    rs = np.random.RandomState(seed)
    for d in ('test', 'attributes'):
        os.makedirs(os.path.join(root, d), exist_ok=True)
    caps = [[int(t) for t in rs.randint(1, words, size=int(rs.randint(3, 25)))] for _ in range(n_img * cpi)]
    ixtoword = {i: 'w%d' % i for i in range(words)}
    with open(os.path.join(root, 'captions.pickle'), 'wb') as f:
        pickle.dump([caps, caps, ixtoword, {v: k for k, v in ixtoword.items()}], f, protocol=2)
    attrs = [[[int(t) for t in rs.randint(1, words, size=int(rs.randint(1, 8)))] for _ in range(int(rs.randint(1, 5)))]
             for _ in range(n_img * cpi)]
    with open(os.path.join(root, 'attributes', 'EE-GAN.pickle'), 'wb') as f:
        pickle.dump([attrs, attrs], f, protocol=2)
    with open(os.path.join(root, 'test', 'filenames.pickle'), 'wb') as f:
        pickle.dump(['t%d' % i for i in range(n_img)], f, protocol=2)
    with open(os.path.join(root, 'test', 'class_info.pickle'), 'wb') as f:
        pickle.dump([1 + i % 3 for i in range(n_img)], f, protocol=2)
    return words


def _save_image_u8(img):
    """vutils.save_image(img, normalize=True, scale_each=True)'s uint8 (miscc/utils.py:11-15) of one
    CHW fp32 image on the host: norm_ip (clamp, - lo, x (1 / max(hi - lo, 1e-5)) -- torch's CUDA
    division by a scalar), then mul(255).add_(0.5).clamp_(0, 255).to(uint8)."""
    x = img.numpy().astype(np.float32)
    lo, hi = float(x.min()), float(x.max())
    inv = np.float32(1.0) / np.float32(max(hi - lo, 1e-5))
    x = np.clip(x, np.float32(lo), np.float32(hi))
    x = (x - np.float32(lo)).astype(np.float32) * inv
    x = (x.astype(np.float32) * np.float32(255)).astype(np.float32) + np.float32(0.5)
    return np.clip(x.astype(np.float32), 0, 255).astype(np.uint8).transpose(1, 2, 0)


def _fid_networks(gpu, n_words, W=8, seed=40):
    import models
    import DAMSM
    from sync_batchnorm import DataParallelWithCallback
    G, A = models.Gen(W, 100), models.ATTR_Enhance()
    T = DAMSM.RNN_ENCODER(n_words, nhidden=256)
    for i, m in enumerate((G, A, T)):
        m.load_state_dict(seeded_state([(k, tuple(v.shape)) for k, v in m.state_dict().items()], seed + i))
    # non-zero residual gains / modulation heads, so every block shapes the image
    with torch.no_grad():
        for n, p in list(G.named_parameters()) + list(A.named_parameters()):
            if n.endswith('gamma'):
                p.fill_(0.5)
    return DataParallelWithCallback(G.to(gpu)), torch.nn.DataParallel(A.to(gpu)), T.to(gpu)


def test_fid_samples_match_host_path(gpu, tmp_path):
    """§8(f)4 sample side (test.py:244-304): the device path -- captions ->
    text encoder -> ATTR_Enhance -> Gen (eval) -> save_image's normalise /
    uint8 -> PIL Resize((299, 299)) -> Inception -> fp64 mu / sigma -- against
    the reference's host arithmetic on the SAME generated images: the resized
    uint8 images equal PIL's bit for bit, the Inception inputs equal the
    reference's ToTensor -> InceptionV3.preprocess of them, and mu / sigma
    equal np.mean / np.cov of the host-path activations (JPEG codec skipped;
    FID values parity-unpinned: random weights)."""
    from PIL import Image
    from datasets import TextOnlyDataset
    from metrics.FID.sampling import SampleGenerator, samples_to_inception_input, fid_of_checkpoints
    from metrics.FID.fid_score import MeasureFID
    words = _text_only_dataset(str(tmp_path))
    netG, attr, enc = _fid_networks(gpu, words)
    ds = TextOnlyDataset(str(tmp_path), 'test')
    sampler = SampleGenerator(netG, attr, enc, ds, batch_size=4, device=gpu)
    model, _ = _seeded_inception(gpu)
    mu, sigma, imgs = sampler.statistics(model, sampling_nums=8, keep_images=True)
    assert imgs.shape == (8, 3, 256, 256) and torch.isfinite(imgs).all()
    # host path on the same images (imgs: the generator's bf16 values)
    u8 = np.stack([np.asarray(Image.fromarray(_save_image_u8(im), 'RGB').resize((299, 299), Image.BILINEAR))
                   for im in imgs])
    from eegan_hip.functional import ImageToNhwcFn
    x = ImageToNhwcFn.apply(imgs.to(gpu))   # bf16 NHWC: exact (the values came from bf16)
    got_u8 = torch.empty((8, 299, 299, 3), dtype=torch.uint8, device=gpu)
    prep = samples_to_inception_input(x, model, u8_out=got_u8)
    d = np.abs(got_u8.cpu().numpy().astype(int) - u8.astype(int))
    print('FID samples: resized uint8 max |device - PIL| = %d' % d.max())
    assert d.max() == 0
    ref_prep = model.preprocess(torch.from_numpy(u8).permute(0, 3, 1, 2).float().div(255).to(gpu))
    assert torch.equal(prep.float(), ref_prep.float())
    host_act = MeasureFID.calculate_activation_statistics(
        [torch.from_numpy(u8).permute(0, 3, 1, 2).float().div(255)], model, verbose=False)
    hmu, hsig = np.mean(host_act, axis=0), np.cov(host_act, rowvar=False)
    emu = np.abs(mu - hmu).max() / np.abs(hmu).max()
    esig = np.abs(sigma - hsig).max() / np.abs(hsig).max()
    print('FID samples: device vs host statistics: mu %.2e sigma %.2e (relative max)' % (emu, esig))
    assert emu <= 1e-10 and esig <= 1e-10
    # one call, two checkpoints' worth of state dicts: its own statistics give FID ~ 0, another ckpt > 0
    sd0 = ({k: v.clone() for k, v in netG.state_dict().items()}, {k: v.clone() for k, v in attr.state_dict().items()})
    sd1 = ({k: (v * 1.5 if v.is_floating_point() and 'running' not in k else v.clone())
            for k, v in sd0[0].items()}, sd0[1])
    fids, stats = fid_of_checkpoints(sampler, [sd0, sd1], (mu, sigma), model=model, sampling_nums=8,
                                     return_stats=True)
    print('FID of two checkpoints vs checkpoint 0 statistics (parity unpinned, 8 samples):', fids)
    # the same captions and noise for every checkpoint: checkpoint 0 reproduces the first call bit for bit
    assert np.array_equal(stats[0][0], mu) and np.array_equal(stats[0][1], sigma)
    assert not np.array_equal(stats[1][0], mu)
    assert all(np.isfinite(f) for f in fids) and fids[0] < fids[1], fids
