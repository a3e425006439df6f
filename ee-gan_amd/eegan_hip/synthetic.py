"""Synthetic device-resident batches with the shapes/distributions of the
reference data pipeline (datasets.py:192-445 via train.py:58-88), used by
bench.py: images U(-1,1) at 64/128/256 (NHWC bf16), captions (B,20) int64
tokens U[1,n_words) with lengths U[5,18] zero-padded, attributes (B,3,5) with
lengths U[1,5], unpaired captions, class ids U[1,class_num].  class_num 0
(MS-COCO: no class_info.pickle, so every image is its own class --
datasets.py:287-295 falls back to np.arange) gives distinct ids, offset by
`id_offset` (rank * B on a data-parallel rank)."""
import torch

from . import functional as Fn


def make_batch(B, device, seed=3407, n_words=5450, words_num=20, class_num=200, attr_num=3, attr_len=5,
               sizes=(64, 128, 256), with_class=True, id_offset=0):
    g = torch.Generator(device='cpu')
    g.manual_seed(seed)
    imgs = []
    for s in sizes:
        x = torch.rand((B, 3, s, s), generator=g) * 2 - 1
        imgs.append(Fn.ImageToNhwcFn.apply(x.to(device)))
    cap_lens = torch.randint(5, 19, (B,), generator=g)
    caps = torch.randint(1, n_words, (B, words_num), generator=g) * (torch.arange(words_num)[None] < cap_lens[:, None])
    attrs_len = torch.randint(1, attr_len + 1, (B, attr_num), generator=g)
    attrs = torch.randint(1, n_words, (B, attr_num, attr_len), generator=g)
    attrs = attrs * (torch.arange(attr_len)[None, None] < attrs_len[..., None])
    un_lens = torch.randint(5, 19, (B,), generator=g)
    un = torch.randint(1, n_words, (B, words_num), generator=g) * (torch.arange(words_num)[None] < un_lens[:, None])
    batch = {
        'imgs': imgs,
        'caps': caps.to(device), 'cap_lens': cap_lens.to(device), 'max_len': int(cap_lens.max()),
        'attrs': attrs.to(device), 'attrs_len': attrs_len.to(device),
        'unpair_caps': un.to(device), 'unpair_cap_lens': un_lens.to(device),
    }
    if with_class:
        if class_num > 0:
            batch['cls_ids'] = torch.randint(1, class_num + 1, (B,), generator=g).to(device)
        else:
            batch['cls_ids'] = (torch.arange(B) + id_offset).to(device)
    return batch
