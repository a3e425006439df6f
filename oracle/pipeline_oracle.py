"""CPU restatement of the reference's image transform chain (TEST
INFRASTRUCTURE ONLY: imported by tests/ and tests/golden/make_pipeline_golden.py,
never by the product).

TextDataset.get_imgs (reference datasets.py:391-424) under train.py's transform
(train.py:269-272) on a PIL image:

    bbox crop (datasets.py:402-410) -> Resize(304) -> RandomCrop(256)
    -> RandomHorizontalFlip -> [Resize(64), Resize(128), itself]
    -> ToTensor -> Normalize((0.5,)*3, (0.5,)*3)

The torchvision transforms (absent from this image; the reference pins no
version) are restated from their published definitions (torchvision >= 0.8):
Resize(int) on a PIL image = PIL `Image.resize((new_w, new_h), BILINEAR)` with
the shorter side -> size and the longer int(size * long / short)
(`_compute_resized_output_size`); RandomCrop.get_params draws
i = torch.randint(0, h - th + 1), then j = torch.randint(0, w - tw + 1) (no
draw when the image already is th x tw); RandomHorizontalFlip draws
torch.rand(1) < 0.5 after the crop; ToTensor = uint8 HWC -> float CHW / 255;
Normalize = (x - 0.5) / 0.5.  Parity of these restatements with a specific
torchvision release is unpinned; PIL (12.2.0 here) is the library they call.
"""
import numpy as np
import torch
from PIL import Image


class TVResize(object):
    def __init__(self, size):
        self.size = size

    def __call__(self, img):
        w, h = img.size
        short, long = (w, h) if w <= h else (h, w)
        new_short, new_long = self.size, int(self.size * long / short)
        new_w, new_h = (new_short, new_long) if w <= h else (new_long, new_short)
        if (new_w, new_h) == (w, h):
            return img
        return img.resize((new_w, new_h), Image.BILINEAR)


class TVRandomCrop(object):
    def __init__(self, size, generator=None):
        self.size, self.g = size, generator

    def __call__(self, img):
        w, h = img.size
        th = tw = self.size
        if w == tw and h == th:
            i = j = 0
        else:
            i = int(torch.randint(0, h - th + 1, size=(1,), generator=self.g).item())
            j = int(torch.randint(0, w - tw + 1, size=(1,), generator=self.g).item())
        self.last = (i, j)
        return img.crop((j, i, j + tw, i + th))


class TVRandomHorizontalFlip(object):
    def __init__(self, p=0.5, generator=None):
        self.p, self.g = p, generator

    def __call__(self, img):
        self.last = bool(torch.rand(1, generator=self.g).item() < self.p)
        return img.transpose(Image.FLIP_LEFT_RIGHT) if self.last else img


class TVCompose(object):
    def __init__(self, ts):
        self.transforms = ts

    def __call__(self, img):
        for t in self.transforms:
            img = t(img)
        return img


def to_tensor_normalize(img):
    """ToTensor + Normalize((0.5,)*3, (0.5,)*3) on the CPU."""
    a = torch.from_numpy(np.array(img, np.uint8, copy=True))
    t = a.view(img.size[1], img.size[0], 3).permute(2, 0, 1).contiguous().to(torch.float32).div(255)
    m = torch.tensor([0.5, 0.5, 0.5])
    return t.sub(m[:, None, None]).div(m[:, None, None])


def train_transform(imsize=256, generator=None):
    """train.py:269-272."""
    crop = TVRandomCrop(imsize, generator)
    flip = TVRandomHorizontalFlip(0.5, generator)
    return TVCompose([TVResize(int(imsize * 76 / 64)), crop, flip]), crop, flip


def get_imgs(rgb, bbox, imsize=(64, 128, 256), generator=None):
    """datasets.py:391-424 on a decoded RGB uint8 array: returns (list of
    normalised CHW fp32 tensors, list of uint8 HWC arrays, (i, j, flip))."""
    img = Image.fromarray(np.asarray(rgb, dtype=np.uint8), 'RGB')
    width, height = img.size
    if bbox is not None:
        r = int(np.maximum(bbox[2], bbox[3]) * 0.75)
        center_x = int((2 * bbox[0] + bbox[2]) / 2)
        center_y = int((2 * bbox[1] + bbox[3]) / 2)
        y1 = np.maximum(0, center_y - r)
        y2 = np.minimum(height, center_y + r)
        x1 = np.maximum(0, center_x - r)
        x2 = np.minimum(width, center_x + r)
        img = img.crop([x1, y1, x2, y2])
    tf, crop, flip = train_transform(imsize[-1], generator)
    img = tf(img)
    ret, raw = [], []
    for i in range(len(imsize)):
        re_img = img if i == len(imsize) - 1 else TVResize(imsize[i])(img)
        raw.append(np.array(re_img, np.uint8))
        ret.append(to_tensor_normalize(re_img))
    return ret, raw, (crop.last[0], crop.last[1], flip.last)


def pil_resize_u8(rgb, out_w, out_h):
    """PIL's bilinear resize of a uint8 RGB array (the oracle of the weight math)."""
    img = Image.fromarray(np.asarray(rgb, dtype=np.uint8), 'RGB')
    return np.array(img.resize((out_w, out_h), Image.BILINEAR), np.uint8)
