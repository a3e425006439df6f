"""FID of the reference (metrics/FID/fid_score.py:50-228) with the feature
network and the activation statistics on the GPU.

  * InceptionV3 pool_3 features: metrics.FID.inception (HIP conv trunk);
  * mu / sigma: eegan_fid_stats (fp64, deterministic) on the device-resident
    activations, instead of copying them to a float64 numpy array and calling
    np.mean / np.cov (fid_score.py:126-127, 183);
  * the Frechet distance: the reference's numpy / scipy.linalg.sqrtm code path
    on the host (fid_score.py:189-228), as there -- O(D^3) once per evaluation.

MeasureFID keeps the reference's static methods (calculate_activation_statistics
returns the N x dims float64 activations as there; calculate_frechet_distance)
and adds activation_statistics (the device path) and statistics_of_images for
image batches already in memory (e.g. generator samples mapped to [0, 1]),
which skips the reference's JPEG round trip through disk.
"""
import os

import numpy as np
import torch
from scipy import linalg

from eegan_hip._lib import ops
from eegan_hip.tensor import stream, workspace

from .inception import InceptionV3


def get_filenames(data_path):
    """miscc/utils.py:76-86, what img_data.Dataset lists (img_data.py:17-20):
    os.walk order (subfolders included, not sorted), every regular file whose
    name contains 'jpg' or 'png' anywhere -- so the image set, its order and
    the batches drop_last removes match the reference's."""
    filenames = []
    for path, _subdirs, files in os.walk(data_path):
        for name in files:
            if name.rfind('jpg') != -1 or name.rfind('png') != -1:
                filename = os.path.join(path, name)
                if os.path.isfile(filename):
                    filenames.append(filename)
    return filenames


def _batches(images):
    for b in images:
        yield b[0] if isinstance(b, (list, tuple)) else b


class MeasureFID(object):

    def __init__(self, model_path=None, dims=2048, batch_size=64, device='cuda'):
        self.model_path, self.dims, self.batch_size = model_path, dims, batch_size
        self.device = torch.device(device)

    def model(self):
        m = InceptionV3(self.model_path, [InceptionV3.BLOCK_INDEX_BY_DIM[self.dims]])
        return m.to(self.device)

    @staticmethod
    def _features(model, batch, device):
        pred = model(batch.to(device))[0]
        if pred.shape[2] != 1 or pred.shape[3] != 1:   # fid_score.py:177-179
            pred = torch.nn.functional.adaptive_avg_pool2d(pred, output_size=(1, 1))
        return pred.reshape(pred.shape[0], -1)

    @staticmethod
    def _features_prepared(model, x):
        """_features on an input already in Inception's NHWC bf16 layout
        (metrics.FID.sampling.samples_to_inception_input)."""
        pred = model.forward_prepared(x)[0]
        if pred.shape[2] != 1 or pred.shape[3] != 1:
            pred = torch.nn.functional.adaptive_avg_pool2d(pred, output_size=(1, 1))
        return pred.reshape(pred.shape[0], -1)

    @staticmethod
    def calculate_activation_statistics(images, model, batch_size=64, dims=2048, cuda=True, verbose=True):
        """fid_score.py:130-187: the pool_3 activations of every batch of
        `images` (an iterable of (B, 3, H, W) [0, 1] batches) as an N x dims
        float64 numpy array."""
        device = next(model.parameters()).device
        preds = [MeasureFID._features(model, b, device) for b in _batches(images)]
        if verbose:
            print(' done')
        return torch.cat(preds).double().cpu().numpy()

    @staticmethod
    def activation_statistics(images, model):
        """(mu, sigma) of the pool_3 activations, computed on the GPU in fp64
        (np.mean / np.cov(rowvar=False) semantics); returned as numpy arrays."""
        device = next(model.parameters()).device
        act = torch.cat([MeasureFID._features(model, b, device) for b in _batches(images)]).contiguous()
        return MeasureFID.device_statistics(act)

    @staticmethod
    def device_statistics(act):
        """mu, sigma of an (N, D) fp32 device tensor of activations."""
        act = act.float().contiguous()
        N, D = act.shape
        mu = torch.empty(D, dtype=torch.float64, device=act.device)
        sigma = torch.empty((D, D), dtype=torch.float64, device=act.device)
        ws = workspace(ops.fid_stats_workspace(D), act.device)
        ops.fid_stats(act.data_ptr(), N, D, mu.data_ptr(), sigma.data_ptr(), ws.data_ptr(), stream())
        return mu.cpu().numpy(), sigma.cpu().numpy()

    def statistics_of_images(self, images, model=None):
        return self.activation_statistics(images, model if model is not None else self.model())

    def calculate_statistic_one(self, given_path, model):
        """fid_score.py:110-128: precomputed .npz statistics, or a folder of
        images read as the reference's img_data.Dataset does (PIL, Resize((299,
        299)), ToTensor) and run through the GPU statistics."""
        if given_path.endswith('.npz'):
            with np.load(given_path) as f:
                return f['mu'][:], f['sigma'][:]
        from PIL import Image
        files = get_filenames(given_path)

        def batches():
            for i in range(0, len(files) - self.batch_size + 1, self.batch_size):   # drop_last=True
                arrs = [np.asarray(Image.open(p).convert('RGB').resize((299, 299), Image.BILINEAR), np.uint8)
                        for p in files[i:i + self.batch_size]]
                yield torch.from_numpy(np.stack(arrs)).permute(0, 3, 1, 2).float().div(255)
        return self.activation_statistics(batches(), model)

    @staticmethod
    def calculate_frechet_distance(mu1, sigma1, mu2, sigma2, eps=1e-6):
        """fid_score.py:189-228: d^2 = |mu1 - mu2|^2 + Tr(C1) + Tr(C2) - 2 Tr(sqrt(C1 C2)),
        with the reference's fallbacks: eps on the diagonals when the product's
        square root is not finite, the real part when the imaginary one is
        negligible (|diag| <= 1e-3), else an error."""
        m1, m2 = np.atleast_1d(mu1), np.atleast_1d(mu2)
        c1, c2 = np.atleast_2d(sigma1), np.atleast_2d(sigma2)
        if m1.shape != m2.shape or c1.shape != c2.shape:
            raise ValueError('statistics of different dimensions: %s / %s' % (m1.shape, m2.shape))
        root, _ = linalg.sqrtm(c1.dot(c2), disp=False)
        if not np.isfinite(root).all():
            print('fid calculation produces singular product; adding %s to diagonal of cov estimates' % eps)
            jitter = np.eye(c1.shape[0]) * eps
            root = linalg.sqrtm((c1 + jitter).dot(c2 + jitter))
        if np.iscomplexobj(root):
            if np.abs(np.diagonal(root).imag).max() > 1e-3:
                raise ValueError('Imaginary component {}'.format(np.abs(root.imag).max()))
            root = root.real
        d = m1 - m2
        return d.dot(d) + np.trace(c1) + np.trace(c2) - 2 * np.trace(root)
