"""Device-side image transform of the training input pipeline.

Replaces the per-image PIL work of TextDataset.get_imgs
(reference datasets.py:391-424) under train.py's transform
(train.py:269-272):

    Resize(int(256 * 76 / 64) = 304) -> RandomCrop(256) -> RandomHorizontalFlip()
    -> [Resize(64), Resize(128), the crop itself] -> ToTensor -> Normalize(0.5, 0.5)

for a whole batch in four HIP launches (csrc/pipeline.hip, eegan_pipe_transform).
The host decodes the JPEGs (PIL, as the reference) and applies the bounding-box
crop arithmetic; everything from the resize on runs on the GPU.

Bit-exactness: torchvision's Resize on a PIL image is PIL's bilinear resample.
The weights are computed here exactly as PIL's Resample.c computes them
(precompute_coeffs + normalize_coeffs_8bpc: support-scaled triangle filter in
double precision, normalised, rounded to 22-bit fixed point), the kernels do
PIL's integer arithmetic (horizontal pass first, uint8 between the passes), so
the uint8 images equal PIL's; ToTensor + Normalize is the same IEEE fp32
arithmetic as torch on the CPU.  The random draws follow torchvision's order
(RandomCrop.get_params: i = randint(0, h - 256 + 1), j = randint(0, w - 256 + 1);
RandomHorizontalFlip: rand(1) < 0.5) on a torch.Generator given by the caller.
"""
import ctypes
import math

import numpy as np
import torch

from ._lib import ops, ImgJob, ScaleTable
from .tensor import empty_nhwc, stream, workspace

PRECISION_BITS = 22


def pil_bilinear_coeffs(in_size, out_size, in0=0.0, in1=None):
    """PIL's bilinear resample weights for one axis (Resample.c,
    precompute_coeffs + normalize_coeffs_8bpc): returns (bounds int32
    [out_size, 2] = (first input index, count), coef int32 [out_size, ksize],
    ksize).  The arithmetic runs in the same order in IEEE double."""
    in1 = float(in_size) if in1 is None else float(in1)
    scale = filterscale = float(np.float32(in1) - np.float32(in0)) / out_size
    if filterscale < 1.0:
        filterscale = 1.0
    support = 1.0 * filterscale                   # bilinear filter support 1.0
    ksize = int(math.ceil(support)) * 2 + 1
    xx = np.arange(out_size, dtype=np.float64)
    center = float(in0) + (xx + 0.5) * scale
    ss = 1.0 / filterscale
    xmin = np.trunc(center - support + 0.5).astype(np.int64)   # C (int) cast
    xmin = np.maximum(xmin, 0)
    xmax = np.trunc(center + support + 0.5).astype(np.int64)
    xmax = np.minimum(xmax, in_size) - xmin
    k = np.zeros((out_size, ksize), dtype=np.float64)
    ww = np.zeros(out_size, dtype=np.float64)
    for x in range(ksize):
        arg = (((x + xmin).astype(np.float64) - center) + 0.5) * ss
        a = np.abs(arg)
        w = np.where(a < 1.0, 1.0 - a, 0.0)
        w = np.where(x < xmax, w, 0.0)
        k[:, x] = w
        ww = ww + w                                # sequential, in x order, as ww += w
    nz = ww != 0.0
    k[nz] = k[nz] / ww[nz, None]
    scaled = k * float(1 << PRECISION_BITS)
    coef = np.where(k < 0, np.trunc(-0.5 + scaled), np.trunc(0.5 + scaled)).astype(np.int32)
    bounds = np.stack([xmin, xmax], 1).astype(np.int32)
    return bounds, coef, ksize


def resized_size(w, h, size):
    """torchvision Resize(int) output (w, h): the shorter side becomes `size`,
    the longer int(size * long / short) (_compute_resized_output_size)."""
    if w <= h:
        return size, int(size * h / w)
    return int(size * w / h), size


def bbox_crop_box(width, height, bbox):
    """The bounding-box crop of get_imgs (datasets.py:400-410) as a box (x1, y1, x2, y2)."""
    if bbox is None:
        return 0, 0, width, height
    r = int(np.maximum(bbox[2], bbox[3]) * 0.75)
    center_x = int((2 * bbox[0] + bbox[2]) / 2)
    center_y = int((2 * bbox[1] + bbox[3]) / 2)
    y1 = int(np.maximum(0, center_y - r))
    y2 = int(np.minimum(height, center_y + r))
    x1 = int(np.maximum(0, center_x - r))
    x2 = int(np.minimum(width, center_x + r))
    return x1, y1, x2, y2


def draw_crop_flip(h, w, crop, generator):
    """torchvision RandomCrop.get_params + RandomHorizontalFlip, in their order."""
    if h < crop or w < crop:
        raise ValueError('Required crop size %d is larger than the input image %dx%d' % (crop, h, w))
    if h == crop and w == crop:
        i = j = 0
    else:
        i = int(torch.randint(0, h - crop + 1, size=(1,), generator=generator).item())
        j = int(torch.randint(0, w - crop + 1, size=(1,), generator=generator).item())
    flip = bool(torch.rand(1, generator=generator).item() < 0.5)
    return i, j, flip


def plan_draws(records, imsize, generator, resize=None):
    """The crop / flip draws of a batch, per record in order (host only): the
    bounding-box crop, Resize(resize) sizes and draw_crop_flip on each."""
    resize = int(imsize * 76 / 64) if resize is None else resize
    out = []
    for arr, bbox in records:
        H, W = np.asarray(arr).shape[:2]
        x1, y1, x2, y2 = bbox_crop_box(W, H, bbox)
        nw, nh = resized_size(x2 - x1, y2 - y1, resize)
        out.append(draw_crop_flip(nh, nw, imsize, generator))
    return out


class DeviceImageTransform(object):
    """Batch transform on the GPU.  __call__(records, generator) takes a list of
    (uint8 HxWx3 array, bbox or None) and returns the list of images per scale
    (ascending), as NHWC bf16 activations (layout 'nhwc_bf16', what the drop-in
    models consume) or the reference's NCHW fp32 tensors ('nchw_f32'), plus the
    draws [(i, j, flip)] per image."""

    def __init__(self, device, imsize=256, base_size=64, branch_num=3, resize=None, layout='nhwc_bf16'):
        self.device = torch.device(device)
        self.crop = imsize
        self.resize = int(imsize * 76 / 64) if resize is None else resize   # train.py:270
        self.scales = [base_size * (2 ** i) for i in range(branch_num)]
        if self.scales[-1] != imsize:
            raise ValueError('the largest scale must be the crop size')
        if layout not in ('nhwc_bf16', 'nchw_f32'):
            raise ValueError(layout)
        self.layout = layout
        self._tables = []
        for s in self.scales[:-1]:
            b, c, k = pil_bilinear_coeffs(imsize, s)
            bt = torch.from_numpy(b.reshape(-1)).to(self.device)
            ct = torch.from_numpy(c.reshape(-1)).to(self.device)
            self._tables.append((s, k, bt, ct))

    def plan(self, records, generator, draws=None):
        """Host side: crop boxes, resize sizes, draws (from `generator`, or the
        given per-record `draws`), PIL weights and the packed source
        sub-rectangles each image's kernels read."""
        given = draws
        if given is not None and len(given) != len(records):
            raise ValueError('%d draws for %d records' % (len(given), len(records)))
        jobs, coefs, bounds, draws, srcs = [], [], [], [], []
        cof = bof = 0
        src_off = 0
        crop = self.crop
        for arr, bbox in records:
            arr = np.asarray(arr)
            if arr.dtype != np.uint8 or arr.ndim != 3 or arr.shape[2] != 3:
                raise ValueError('records hold uint8 HxWx3 RGB arrays')
            H, W = arr.shape[:2]
            x1, y1, x2, y2 = bbox_crop_box(W, H, bbox)
            cw, ch = x2 - x1, y2 - y1
            nw, nh = resized_size(cw, ch, self.resize)
            if given is None:
                i, j, flip = draw_crop_flip(nh, nw, crop, generator)
            else:
                i, j, flip = (int(given[len(draws)][0]), int(given[len(draws)][1]), bool(given[len(draws)][2]))
                if not (0 <= i <= nh - crop and 0 <= j <= nw - crop):
                    raise ValueError('crop draw (%d, %d) outside the %dx%d resized image' % (i, j, nh, nw))
            draws.append((i, j, flip))
            hb, hc, hk = pil_bilinear_coeffs(cw, nw)
            vb, vc, vk = pil_bilinear_coeffs(ch, nh)
            hb, hc = hb[j:j + crop].copy(), hc[j:j + crop]
            vb, vc = vb[i:i + crop].copy(), vc[i:i + crop]
            # the source sub-rectangle the crop window's supports touch
            c0, c1 = int(hb[0, 0]), int(hb[-1, 0] + hb[-1, 1])
            r0, r1 = int(vb[0, 0]), int(vb[-1, 0] + vb[-1, 1])
            sub = np.ascontiguousarray(arr[y1 + r0:y1 + r1, x1 + c0:x1 + c1])
            hb[:, 0] -= c0
            vb[:, 0] -= r0
            jobs.append((src_off, sub.shape[1] * 3, 0, r1 - r0, int(flip), cof, bof, hk,
                         cof + hc.size, bof + hb.size, vk))
            coefs += [hc.reshape(-1), vc.reshape(-1)]
            bounds += [hb.reshape(-1), vb.reshape(-1)]
            cof += hc.size + vc.size
            bof += hb.size + vb.size
            srcs.append(sub)
            src_off += (sub.nbytes + 15) // 16 * 16
        return jobs, np.concatenate(coefs), np.concatenate(bounds), draws, srcs, src_off

    def __call__(self, records, generator, crop_u8=None, draws=None):
        B = len(records)
        jobs, coef, bounds, draws, srcs, nsrc = self.plan(records, generator, draws)
        dev = self.device
        host = torch.empty(nsrc, dtype=torch.uint8, pin_memory=torch.cuda.is_available())
        hv = host.numpy()
        for (off, *_), sub in zip(jobs, srcs):
            hv[off:off + sub.nbytes] = sub.reshape(-1)
        src = host.to(dev, non_blocking=True)
        jarr = (ImgJob * B)(*[ImgJob(*j) for j in jobs])
        jt = torch.frombuffer(bytearray(bytes(jarr)), dtype=torch.uint8).to(dev)
        ct = torch.from_numpy(coef).to(dev)
        bt = torch.from_numpy(bounds).to(dev)
        max_rows = max(j[3] for j in jobs)
        crop = self.crop
        sizes = (ctypes.c_int * len(self.scales))(*self.scales)
        ws = workspace(ops.pipe_workspace(B, crop, max_rows, len(self.scales), sizes), dev)
        tabs = (ScaleTable * len(self.scales))()
        for t, (s, k, b_, c_) in zip(tabs, self._tables):
            t.size, t.ksize = s, k
            t.hcoef = t.vcoef = c_.data_ptr()
            t.hbounds = t.vbounds = b_.data_ptr()
        tabs[len(self.scales) - 1].size = crop
        outs = []
        for s in self.scales:
            if self.layout == 'nhwc_bf16':
                outs.append(empty_nhwc(B, 3, s, s, dev))
            else:
                outs.append(torch.empty((B, 3, s, s), dtype=torch.float32, device=dev))
        PA = ctypes.c_void_p * len(self.scales)
        ptrs = PA(*[o.data_ptr() for o in outs])
        f32 = ptrs if self.layout == 'nchw_f32' else None
        bf = ptrs if self.layout == 'nhwc_bf16' else None
        ops.pipe_transform(src.data_ptr(), jt.data_ptr(), B, max_rows, crop, ct.data_ptr(), bt.data_ptr(),
                           len(self.scales), tabs, f32, bf, 8 if bf is not None else 0,
                           crop_u8.data_ptr() if crop_u8 is not None else None, ws.data_ptr(), stream())
        return outs, draws
