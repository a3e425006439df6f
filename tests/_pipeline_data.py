"""A small synthetic dataset in the reference's on-disk layout (datasets.py:
filenames.pickle per split, captions.pickle, attributes/EE-GAN.pickle,
class_info.pickle, bounding_boxes.pickle, images/<key>.jpg), generated from a
seed so tests/golden/make_pipeline_golden.py and the tests build identical
files.  Images are stored losslessly (PNG bytes under the .jpg name -- PIL opens
by content), so the decoded pixels are the generated ones."""
import os
import pickle

import numpy as np

# (width, height) per image: upscaled (< 304 short side), downscaled, square,
# portrait / landscape, bbox crops touching the borders
SIZES = [(150, 110), (420, 330), (333, 500), (304, 304), (260, 380), (500, 297)]
WORDS = 60
CAPS_PER_IMAGE = 10


def image(k, w, h):
    rs = np.random.RandomState(1000 + k)
    base = rs.randint(0, 256, size=(h // 8 + 2, w // 8 + 2, 3)).astype(np.float64)
    # smooth-ish content with fine noise (resampling differences show up)
    yy = (np.arange(h) / 8.0)[:, None]
    xx = (np.arange(w) / 8.0)[None, :]
    y0, x0 = yy.astype(int), xx.astype(int)
    fy, fx = (yy - y0)[..., None], (xx - x0)[..., None]
    img = (base[y0, x0] * (1 - fy) * (1 - fx) + base[y0 + 1, x0] * fy * (1 - fx) +
           base[y0, x0 + 1] * (1 - fy) * fx + base[y0 + 1, x0 + 1] * fy * fx)
    img += rs.randint(-20, 21, size=img.shape)
    return np.clip(img, 0, 255).astype(np.uint8)


def bboxes():
    out = {}
    for k, (w, h) in enumerate(SIZES):
        rs = np.random.RandomState(2000 + k)
        bw, bh = int(rs.randint(w // 3, w)), int(rs.randint(h // 3, h))
        out['img%d' % k] = [int(rs.randint(0, w - bw + 1)), int(rs.randint(0, h - bh + 1)), bw, bh]
    out['img1'] = [0, 0, SIZES[1][0], SIZES[1][1]]        # whole image: crop clamped on every side
    return out


def build(root):
    """Write the dataset under `root` (bird layout); returns the image arrays."""
    rs = np.random.RandomState(7)
    os.makedirs(os.path.join(root, 'images'), exist_ok=True)
    os.makedirs(os.path.join(root, 'train'), exist_ok=True)
    os.makedirs(os.path.join(root, 'attributes'), exist_ok=True)
    from PIL import Image
    keys, arrs = [], []
    for k, (w, h) in enumerate(SIZES):
        key = 'img%d' % k
        a = image(k, w, h)
        Image.fromarray(a, 'RGB').save(os.path.join(root, 'images', key + '.jpg'), format='PNG')
        keys.append(key)
        arrs.append(a)
    n = len(keys)
    # captions: lengths 3..30 (some longer than WORDS_NUM: the random-subset branch)
    caps = [[int(t) for t in rs.randint(1, WORDS, size=int(rs.randint(3, 31)))] for _ in range(n * CAPS_PER_IMAGE)]
    test_caps = caps[:CAPS_PER_IMAGE]
    ixtoword = {i: 'w%d' % i for i in range(WORDS)}
    wordtoix = {v: k for k, v in ixtoword.items()}
    with open(os.path.join(root, 'captions.pickle'), 'wb') as f:
        pickle.dump([caps, test_caps, ixtoword, wordtoix], f, protocol=2)
    # attributes: per caption a list of phrases (0..6 phrases of 0..8 tokens)
    attrs = [[[int(t) for t in rs.randint(1, WORDS, size=int(rs.randint(0, 9)))] for _ in range(int(rs.randint(0, 7)))]
             for _ in range(n * CAPS_PER_IMAGE)]
    with open(os.path.join(root, 'attributes', 'EE-GAN.pickle'), 'wb') as f:
        pickle.dump([attrs, attrs[:CAPS_PER_IMAGE]], f, protocol=2)
    with open(os.path.join(root, 'train', 'filenames.pickle'), 'wb') as f:
        pickle.dump(keys, f, protocol=2)
    with open(os.path.join(root, 'train', 'class_info.pickle'), 'wb') as f:
        pickle.dump([1, 2, 1, 3, 2, 200], f, protocol=2)
    with open(os.path.join(root, 'bounding_boxes.pickle'), 'wb') as f:
        pickle.dump(bboxes(), f, protocol=2)
    return arrs
