"""Input pipeline on the CPU (reference datasets.py:192-445,
train.py:269-272): the oracle's transform chain against the golden vectors
captured from the reference's own TextDataset, the drop-in reader's text
fields against the same vectors, the host-side PIL weight math against PIL
itself, torchvision-order draws, and the restricted unpickler."""
import os
import pickle
import sys

import numpy as np
import pytest
import torch

from _util import REPO

sys.path.insert(0, os.path.join(REPO, 'tests'))
import _pipeline_data as PD  # noqa: E402

GOLD = os.path.join(REPO, 'tests', 'golden', 'pipeline.npz')
SEEDS = [11, 12, 13, 14, 15, 16]


def _golden():
    return np.load(GOLD)


def test_oracle_transform_matches_reference_golden():
    from oracle import pipeline_oracle as PO
    g = _golden()
    bbs = PD.bboxes()
    for idx, (w, h) in enumerate(PD.SIZES):
        p = 's%d/' % idx
        s = int(g[p + 'draws'][0])
        imgs, raws, (i, j, fl) = PO.get_imgs(PD.image(idx, w, h), bbs['img%d' % idx],
                                             generator=torch.Generator().manual_seed(s))
        assert [i, j, int(fl)] == list(g[p + 'draws'][2:]), idx
        sums = [int(r.astype(np.int64).sum()) for r in raws] + \
               [int((r.astype(np.int64) * np.arange(r.size).reshape(r.shape) % 9973).sum()) for r in raws]
        assert sums == list(g[p + 'u8_sums']), idx
        if idx < 3:
            for r in raws:
                assert np.array_equal(r, g[p + 'u8_%d' % r.shape[0]])
        for k, im in zip((64, 128, 256), imgs):
            assert np.array_equal(im.reshape(-1)[:64].numpy(), g[p + 'f32_%d_head' % k])


def test_dropin_reader_text_fields_match_reference(tmp_path):
    """The drop-in TextDataset over the reference's on-disk formats draws the
    same caption / attribute / unpaired caption as the reference under the
    same numpy seed (datasets.py:301-389)."""
    import datasets as DS
    from miscc.config import cfg
    g = _golden()
    PD.build(str(tmp_path))
    words_num, attr_num, attr_len, cpi = [int(v) for v in g['cfg']]
    old = (cfg.TEXT.WORDS_NUM, cfg.TEXT.MAX_ATTR_NUM, cfg.TEXT.MAX_ATTR_LEN, cfg.TEXT.CAPTIONS_PER_IMAGE)
    cfg.TEXT.WORDS_NUM, cfg.TEXT.MAX_ATTR_NUM, cfg.TEXT.MAX_ATTR_LEN = words_num, attr_num, attr_len
    cfg.TEXT.CAPTIONS_PER_IMAGE = cpi
    try:
        ds = DS.TextDataset(str(tmp_path), 'bird')
        assert len(ds) == len(PD.SIZES) and ds.n_words == PD.WORDS
        for idx in range(len(PD.SIZES)):
            p = 's%d/' % idx
            np.random.seed(int(g[p + 'draws'][0]))
            basic, attrs, unpair = ds[idx]
            image, cap, cap_len, cls_id, key = basic
            assert key == bytes(g[p + 'key']).decode()
            assert np.array_equal(np.asarray(cap).reshape(-1), g[p + 'cap'])
            assert [int(cap_len), int(cls_id)] == list(g[p + 'text'])
            assert np.array_equal(np.asarray(attrs[0]).reshape(-1), g[p + 'attrs'])
            assert [int(attrs[1])] + list(np.asarray(attrs[2]).reshape(-1)) == list(g[p + 'attr_num_lens'])
            assert np.array_equal(np.asarray(unpair[0]).reshape(-1), g[p + 'unpair_cap'])
            assert [int(unpair[1]), int(unpair[2])] == list(g[p + 'unpair'])
            w, h = PD.SIZES[idx]
            assert np.array_equal(image.rgb, PD.image(idx, w, h)) and image.bbox == PD.bboxes()[key]
    finally:
        cfg.TEXT.WORDS_NUM, cfg.TEXT.MAX_ATTR_NUM, cfg.TEXT.MAX_ATTR_LEN, cfg.TEXT.CAPTIONS_PER_IMAGE = old


def _emulate_pil(rgb, out_w, out_h):
    """PIL's two-pass integer resample with the product's weight tables."""
    from eegan_hip.pipeline import pil_bilinear_coeffs
    h, w = rgb.shape[:2]

    def one(a, n_out, axis):
        b, c, k = pil_bilinear_coeffs(a.shape[axis], n_out)
        a = np.moveaxis(a.astype(np.int64), axis, 0)
        out = np.empty((n_out,) + a.shape[1:], np.int64)
        for o in range(n_out):
            x0, n = b[o]
            s = np.full(a.shape[1:], 1 << 21, np.int64)
            for t in range(n):
                s += a[x0 + t] * int(c[o, t])
            out[o] = np.clip(s >> 22, 0, 255)   # clip8: >= 2^30 -> 255, <= 0 -> 0
        return np.moveaxis(out, 0, axis).astype(np.uint8)
    tmp = one(rgb, out_w, 1) if out_w != w else rgb
    return one(tmp, out_h, 0) if out_h != h else tmp


@pytest.mark.parametrize('src,dst', [((150, 110), (304, 414)), ((420, 330), (387, 304)), ((333, 500), (304, 456)),
                                     ((256, 256), (64, 64)), ((256, 256), (128, 128)), ((301, 299), (305, 304)),
                                     ((97, 1000), (33, 340))])
def test_pil_weight_math_matches_pil(src, dst):
    from oracle import pipeline_oracle as PO
    rs = np.random.RandomState(src[0] * 7 + dst[1])
    rgb = rs.randint(0, 256, size=(src[1], src[0], 3)).astype(np.uint8)
    got = _emulate_pil(rgb, dst[0], dst[1])
    ref = PO.pil_resize_u8(rgb, dst[0], dst[1])
    assert np.array_equal(got, ref)


def test_draws_follow_torchvision_order():
    from eegan_hip.pipeline import draw_crop_flip
    from oracle import pipeline_oracle as PO
    from PIL import Image
    for s, (w, h) in enumerate([(304, 412), (560, 304), (256, 256), (300, 300)]):
        g1, g2 = torch.Generator().manual_seed(s), torch.Generator().manual_seed(s)
        i, j, fl = draw_crop_flip(h, w, 256, g1)
        img = Image.new('RGB', (w, h))
        crop, flip = PO.TVRandomCrop(256, g2), PO.TVRandomHorizontalFlip(0.5, g2)
        flip(crop(img))
        assert (i, j, fl) == (crop.last[0], crop.last[1], flip.last)


def test_safe_unpickler_refuses_code(tmp_path):
    import datasets as DS
    p = tmp_path / 'evil.pickle'
    with open(p, 'wb') as f:
        pickle.dump(os.system, f)
    with pytest.raises(pickle.UnpicklingError):
        DS.load_pickle(str(p))
    q = tmp_path / 'ok.pickle'
    with open(q, 'wb') as f:
        pickle.dump([{'a': [1, 2]}, np.arange(3), (1.5, 'x')], f, protocol=2)
    v = DS.load_pickle(str(q))
    assert v[0] == {'a': [1, 2]} and np.array_equal(v[1], np.arange(3)) and v[2] == (1.5, 'x')
