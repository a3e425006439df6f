"""Device input pipeline on the MI355X (csrc/pipeline.hip through the C ABI)
against the CPU oracle (oracle/pipeline_oracle.py: the reference's get_imgs
chain over PIL, pinned by tests/golden/pipeline.npz): uint8 crops and 64/128
scales bit-exact, the normalised fp32 tensors bit-exact, the bf16 NHWC
activations equal to their rounding, the crop / flip draws equal to the
seeded host draw, on the reference's sample set and on random batches
(upscaled, downscaled, square, bbox crops clamped at the borders)."""
import os
import sys

import numpy as np
import pytest
import torch

from _util import REPO

sys.path.insert(0, os.path.join(REPO, 'tests'))
import _pipeline_data as PD  # noqa: E402

pytestmark = pytest.mark.gpu


def _check_batch(gpu, records, seed, layout):
    from eegan_hip.pipeline import DeviceImageTransform
    from oracle import pipeline_oracle as PO
    tf = DeviceImageTransform(gpu, layout=layout)
    crop_u8 = torch.empty((len(records), 256, 256, 3), dtype=torch.uint8, device=gpu)
    outs, draws = tf(records, torch.Generator().manual_seed(seed), crop_u8=crop_u8)
    torch.cuda.synchronize()
    g = torch.Generator().manual_seed(seed)
    crop_u8 = crop_u8.cpu().numpy()
    for b, (rgb, bbox) in enumerate(records):
        ref, raws, d = PO.get_imgs(rgb, bbox, generator=g)
        assert tuple(draws[b]) == tuple(d), (b, draws[b], d)
        assert np.array_equal(crop_u8[b], raws[-1]), b
        for k, (o, r) in enumerate(zip(outs, ref)):
            o = o[b].float().cpu() if layout == 'nhwc_bf16' else o[b].cpu()
            r = r.to(torch.bfloat16).float() if layout == 'nhwc_bf16' else r
            assert torch.equal(o, r), (b, k)


@pytest.mark.parametrize('layout', ['nchw_f32', 'nhwc_bf16'])
def test_pipeline_reference_samples(gpu, layout):
    bbs = PD.bboxes()
    recs = [(PD.image(k, w, h), bbs['img%d' % k]) for k, (w, h) in enumerate(PD.SIZES)]
    _check_batch(gpu, recs, 11, layout)


def test_pipeline_random_batch(gpu):
    """32 images of random sizes 80..720 px, random / absent / border bboxes."""
    rs = np.random.RandomState(5)
    recs = []
    for b in range(32):
        w, h = int(rs.randint(80, 721)), int(rs.randint(80, 721))
        rgb = rs.randint(0, 256, size=(h, w, 3)).astype(np.uint8)
        kind = b % 3
        if kind == 0:
            bbox = None
        elif kind == 1:
            bw, bh = int(rs.randint(8, w + 1)), int(rs.randint(8, h + 1))
            bbox = [int(rs.randint(0, w - bw + 1)), int(rs.randint(0, h - bh + 1)), bw, bh]
        else:
            bbox = [0, 0, w, h]
        recs.append((rgb, bbox))
    _check_batch(gpu, recs, 99, 'nchw_f32')


def test_device_dataloader_end_to_end(gpu, tmp_path):
    """DeviceDataLoader over the reference's on-disk formats: the batch has the
    reference's structure, its images equal the oracle's per sample."""
    import datasets as DS
    from oracle import pipeline_oracle as PO
    PD.build(str(tmp_path))
    ds = DS.TextDataset(str(tmp_path), 'bird')
    dl = DS.DeviceDataLoader(ds, 4, gpu, shuffle=False, num_workers=0, seed=21)
    g = torch.Generator().manual_seed(21)
    n = 0
    for basic, attrs, unpair in dl:
        imgs, caps, cap_lens, cls_ids, keys = basic
        assert [tuple(t.shape) for t in imgs] == [(4, 3, 64, 64), (4, 3, 128, 128), (4, 3, 256, 256)]
        assert all(t.is_cuda and t.dtype == torch.float32 for t in imgs)
        from miscc.config import cfg
        assert tuple(caps.shape) == (4, cfg.TEXT.WORDS_NUM, 1) and tuple(cap_lens.shape) == (4,)
        for b, key in enumerate(keys):
            k = int(key[3:])
            w, h = PD.SIZES[k]
            ref, _, _ = PO.get_imgs(PD.image(k, w, h), PD.bboxes()[key], generator=g)
            for t, r in zip(imgs, ref):
                assert torch.equal(t[b].cpu(), r), (key, t.shape)
        n += 1
    assert n == len(PD.SIZES) // 4
