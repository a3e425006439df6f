"""Generated-sample side of the FID leg (reference test.py:187-304 feeding
metrics/FID/fid_score.py:98-228), on the device end to end.

The reference evaluates a checkpoint in two programs: test.py generates one
256 px image per test caption (`traverse_dataset_30k` -> `gen_one_batch_attr`:
text encoder -> ATTR_Enhance -> attr_merge -> Gen, eval mode, no_grad) and
saves each with vutils.save_image(normalize=True, scale_each=True) as a JPEG
(miscc/utils.py:11-15); fid_score.py reads the folder back (PIL,
Resize((299, 299)), ToTensor, img_data.Dataset), runs InceptionV3 and compares
the pool_3 statistics with the dataset's.  Here one call does the whole loop
per checkpoint with nothing leaving the GPU but mu / sigma:

  TextOnlyDataset captions (torch DataLoader, the reference's draws) ->
  RNN_ENCODER (HIP LSTM) -> ATTR_Enhance -> Gen (HIP convs, eval BN) ->
  eegan_fid_samples: per-image min/max normalise, uint8, PIL-exact bilinear
  256 -> 299, ToTensor, Inception renormalisation (one fused pass) ->
  InceptionV3 pool_3 (HIP trunk) -> eegan_fid_stats (fp64 mu / sigma) ->
  Frechet distance on the host (scipy sqrtm, as the reference).

The one step skipped is the JPEG codec of the saved files (lossy; the
statistics of the decoded files differ from the uint8 images by the codec's
error).  FID values are "parity unpinned" here: the pretrained Inception /
DAMSM weights and the datasets are absent, so only the arithmetic is pinned
(tests/test_gpu_fid.py: the device sample path equals the host path --
save_image's arithmetic, PIL's resize, np.mean / np.cov -- on the same
generated images).
"""
import ctypes

import numpy as np
import torch

from eegan_hip._lib import ops
from eegan_hip.pipeline import pil_bilinear_coeffs
from eegan_hip.tensor import empty_nhwc, ld_of, stream, workspace

from .fid_score import MeasureFID
from .inception import InceptionV3

FID_SIZE = 299   # fid_score.py:106 Resize((299, 299))


class _Resample(object):
    """PIL bilinear weights (eegan_hip.pipeline.pil_bilinear_coeffs) for
    H x W -> FID_SIZE^2, resident on the device."""

    def __init__(self, H, W, device):
        hb, hc, hk = pil_bilinear_coeffs(W, FID_SIZE)
        vb, vc, vk = pil_bilinear_coeffs(H, FID_SIZE)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a).reshape(-1)).to(device)  # noqa: E731
        self.hb, self.hc, self.hk = t(hb), t(hc), hk
        self.vb, self.vc, self.vk = t(vb), t(vc), vk


def samples_to_inception_input(img, model, resample=None, u8_out=None):
    """Generator images (NHWC bf16 activations of logical shape (N, 3, H, W),
    values in [-1, 1]) -> the NHWC bf16 Inception input the reference's
    save -> reload -> Resize((299, 299)) -> ToTensor -> InceptionV3.preprocess
    chain produces (JPEG codec aside).  `u8_out` (N, 299, 299, 3) uint8: the
    resized images themselves (tests)."""
    N, C, H, W = img.shape
    if C != 3:
        raise ValueError('3-channel images expected')
    if img.dtype != torch.bfloat16 or img.stride(1) != 1:
        raise ValueError('samples_to_inception_input takes the generator\'s NHWC bf16 images')
    ld = ld_of(img)
    rs = resample if resample is not None else _Resample(H, W, img.device)
    sc, sh = model.input_affine()
    F3 = ctypes.c_float * 3
    y = empty_nhwc(N, 3, FID_SIZE, FID_SIZE, img.device)
    ws = workspace(ops.fid_samples_workspace(N, H, FID_SIZE), img.device)
    ops.fid_samples(img.data_ptr(), N, H, W, ld, FID_SIZE, FID_SIZE, rs.hc.data_ptr(), rs.hb.data_ptr(), rs.hk,
                    rs.vc.data_ptr(), rs.vb.data_ptr(), rs.vk, F3(*sc), F3(*sh), y.data_ptr(), ld_of(y),
                    u8_out.data_ptr() if u8_out is not None else None, ws.data_ptr(), stream())
    return y


def _module(m):
    return getattr(m, 'module', m)


class SampleGenerator(object):
    """test.py's Tester for the FID leg: the networks (netG and attr_enhance as
    train.py saves them, i.e. wrapped, `module.`-prefixed state dicts), the
    frozen text encoder, and a TextOnlyDataset traversed by a torch DataLoader
    (batch_size, shuffle=True, drop_last=True: test.py:124-128)."""

    def __init__(self, netG, attr_enhance, text_encoder, dataset, batch_size, device='cuda', max_attr_num=None,
                 seed=3407, num_workers=0):
        from miscc.config import cfg
        self.netG, self.attr_enhance, self.text_encoder = netG, attr_enhance, text_encoder
        self.dataset, self.batch_size = dataset, batch_size
        self.device = torch.device(device)
        self.max_attr_num = cfg.TEXT.MAX_ATTR_NUM if max_attr_num is None else max_attr_num
        self.seed = seed
        self._shuffle = torch.Generator()   # the loader's permutation, re-seeded per statistics() call
        self.loader = torch.utils.data.DataLoader(dataset, batch_size=batch_size, drop_last=True, shuffle=True,
                                                  num_workers=num_workers, generator=self._shuffle)
        self._resample = None

    def load(self, netG_state, attr_state):
        """One checkpoint (test.py:205-211)."""
        self.netG.load_state_dict(netG_state)
        self.attr_enhance.load_state_dict(attr_state)

    @torch.no_grad()
    def gen_one_batch(self, data, noise):
        """test.py:58-72 prepare_data + 280-300 gen_one_batch_attr -> img256."""
        (caps, cap_lens, _cls, _keys), rev_attrs = data
        dev = self.device
        B = caps.shape[0]
        caps = caps.reshape(B, -1).to(dev)
        cap_lens = cap_lens.reshape(-1).to(dev)
        enc = self.text_encoder
        hidden = enc.init_hidden(B)
        _, sent = enc(caps, cap_lens, hidden)
        attrs, _, attrs_len = rev_attrs
        attrs = attrs.reshape(B, attrs.shape[1], -1).to(dev)
        attrs_len = attrs_len.reshape(B, -1)
        embs = [enc(attrs[:, i, :], attrs_len[:, i].to(dev), hidden)[1] for i in range(self.max_attr_num)]
        attrs_emb = torch.stack(embs, dim=1)
        _, attn = self.attr_enhance(sent, attrs_emb)
        attn = _module(self.attr_enhance).attr_merge(attn)
        return self.netG(noise, sent, attn)[-1]

    @torch.no_grad()
    def statistics(self, model, sampling_nums=30000, generator=None, keep_images=False):
        """mu, sigma of `sampling_nums` generated images (rounded up to whole
        batches, test.py:188-193; one pass over the loader at most, as
        traverse_dataset_30k with repeat_times 1).  generator: a torch.Generator
        on the device for the noise (default: seeded by `seed`)."""
        for m in (self.netG, self.attr_enhance, self.text_encoder):
            m.eval()
        max_iter = -(-sampling_nums // self.batch_size)
        if generator is None:
            generator = torch.Generator(device=self.device).manual_seed(self.seed)
        np_state = np.random.get_state()
        np.random.seed(self.seed)   # the dataset's caption / attribute draws (numpy.random)
        self._shuffle.manual_seed(self.seed)
        feats, kept = [], []
        try:
            for it, data in enumerate(self.loader):
                if it >= max_iter:
                    break
                B = data[0][0].shape[0]
                noise = torch.randn(B, 100, device=self.device, generator=generator)
                img = self.gen_one_batch(data, noise)
                if self._resample is None:
                    self._resample = _Resample(img.shape[2], img.shape[3], self.device)
                x = samples_to_inception_input(img, model, self._resample)
                feats.append(MeasureFID._features_prepared(model, x))
                if keep_images:
                    kept.append(img.float().cpu())
        finally:
            np.random.set_state(np_state)
        if not feats:
            raise ValueError('the loader yielded no batch (dataset smaller than one batch with drop_last)')
        act = torch.cat(feats).contiguous()
        mu, sigma = MeasureFID.device_statistics(act)
        return (mu, sigma, torch.cat(kept)) if keep_images else (mu, sigma)


def fid_of_checkpoints(sampler, checkpoints, ref_stats, model=None, sampling_nums=30000, dims=2048,
                       return_stats=False):
    """FID of each checkpoint (netG_state, attr_enhance_state) against the
    reference statistics (mu, sigma) -- an .npz's or a folder's
    (MeasureFID.calculate_statistic_one) -- the loop of test.py:202-237 over
    select_epochs with fid_score.py's comparison.  Every checkpoint sees the
    same captions and noise.  Returns a list of floats ("parity unpinned"
    without the pretrained weights), and with return_stats the list of each
    checkpoint's (mu, sigma) as well."""
    if model is None:
        model = InceptionV3(None, [InceptionV3.BLOCK_INDEX_BY_DIM[dims]]).to(sampler.device)
    mu_r, sig_r = ref_stats
    out, stats = [], []
    for g_state, a_state in checkpoints:
        sampler.load(g_state, a_state)
        mu, sig = sampler.statistics(model, sampling_nums)
        stats.append((mu, sig))
        out.append(float(MeasureFID.calculate_frechet_distance(mu, sig, mu_r, sig_r)))
    return (out, stats) if return_stats else out
