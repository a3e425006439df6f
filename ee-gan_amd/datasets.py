"""Drop-in `datasets` module (reference datasets.py:36-52, 192-445): the
host-side reader of the reference's on-disk formats and the text-side sample
logic, with the image transform moved to the GPU (eegan_hip.pipeline).

What stays on the host (as in the reference): unpickling the metadata --
filenames.pickle (datasets.py:231-239), bounding_boxes.pickle (242-246),
attributes/<name>.pickle (249-266), captions.pickle (269-284),
class_info.pickle (287-295) -- the caption / attribute / unpaired-caption
draws (numpy.random, 301-389, the reference imports numpy.random as `random`),
JPEG decoding (PIL) and the bounding-box crop arithmetic.  What moves to the
GPU: Resize(304) -> RandomCrop(256) -> RandomHorizontalFlip -> Resize(64/128)
-> ToTensor + Normalize for the whole batch (train.py:269-272,
datasets.py:412-424), bit-exact to PIL / torch on the CPU.

Pickles are read with a restricted unpickler that only rebuilds plain
containers, numbers, strings and numpy arrays (the formats above hold nothing
else); any other global in the file raises instead of being imported.

`TextDataset.__getitem__` returns the reference's nested sample
([image, cap, cap_len, cls_id, key], attrs, unpair) with `image` a
`HostImage` (decoded uint8 RGB + bbox).  Two ways to batch them:

  * train.py's own `torch.utils.data.DataLoader` (train.py:274-278, default
    collate): HostImage registers a collate function, so a batch's `imgs` is a
    `HostImageBatch` -- one entry per scale whose `.to(device)` (train.py:70)
    runs the device transform for the whole batch once; the crop / flip draws
    are taken at collate time from torch's global generator, in the process
    that collates, in torchvision's per-sample order (where the reference's
    transform draws them, datasets.py:412-413);
  * `DeviceDataLoader`: the same, with the draws from its own generator and
    the images in the drop-in models' NHWC bf16 layout if asked.

Data parallel (one process per GPU, eegan_hip.launch): the reference's
DataParallel scatters ONE batch over its GPUs (train.py:220-228).  Under
torchrun every rank runs train.py with the same seed and the same shuffled
DataLoader, so with a process group of world W up (or `shard=(rank, W)`) the
dataset is rank r's stride-W shard -- item i is sample i*W + r, len // W items
on every rank (equal, so every rank runs the same number of steps) -- and the
constructor puts ranks > 0 on random streams of their own
(launch.offset_rank_rngs), so captions, crops and noise differ across ranks.
`--batch_size` is then the per-rank batch.
"""
import io
import os
import pickle

import numpy as np
import numpy.random as random   # the reference's draws (datasets.py:28)
import torch
import torch.utils.data as data

from miscc.config import cfg


# ----------------------------------------------------------------- pickles --
class _SafeUnpickler(pickle.Unpickler):
    _ALLOWED = {
        ('builtins', 'list'), ('builtins', 'dict'), ('builtins', 'set'), ('builtins', 'frozenset'),
        ('builtins', 'tuple'), ('builtins', 'int'), ('builtins', 'float'), ('builtins', 'str'),
        ('builtins', 'bytes'), ('builtins', 'bytearray'), ('builtins', 'complex'), ('builtins', 'bool'),
        ('__builtin__', 'list'), ('__builtin__', 'dict'), ('__builtin__', 'set'), ('__builtin__', 'tuple'),
        ('__builtin__', 'int'), ('__builtin__', 'long'), ('__builtin__', 'float'), ('__builtin__', 'unicode'),
        ('__builtin__', 'str'), ('copy_reg', '_reconstructor'), ('copyreg', '_reconstructor'),
        ('collections', 'OrderedDict'), ('collections', 'defaultdict'),
        ('numpy', 'ndarray'), ('numpy', 'dtype'), ('numpy.core.multiarray', '_reconstruct'),
        ('numpy.core.multiarray', 'scalar'), ('numpy._core.multiarray', '_reconstruct'),
        ('numpy._core.multiarray', 'scalar'), ('_codecs', 'encode'),
    }

    def find_class(self, module, name):
        if (module, name) not in self._ALLOWED:
            raise pickle.UnpicklingError('refusing to load %s.%s from a dataset pickle' % (module, name))
        if module == '__builtin__':
            module = 'builtins'
            name = {'long': 'int', 'unicode': 'str'}.get(name, name)
        return super().find_class(module, name)


def load_pickle(path, encoding='ASCII'):
    with open(path, 'rb') as f:
        return _SafeUnpickler(io.BytesIO(f.read()), encoding=encoding).load()


# ----------------------------------------------------------------- samples --
class HostImage(object):
    """A decoded sample image: uint8 RGB array (H, W, 3) and its bounding box
    (x, y, w, h) or None -- the state of get_imgs (datasets.py:400) before the
    transform, which the device pipeline applies batch-wise -- and the
    dataset's scales (`TextDataset.imsize`; a spawned DataLoader worker's cfg
    holds the defaults, not the YAML train.py loaded)."""
    __slots__ = ('rgb', 'bbox', 'imsize')

    def __init__(self, rgb, bbox, imsize=None):
        self.rgb, self.bbox, self.imsize = rgb, bbox, imsize


def decode_rgb(path):
    from PIL import Image
    with Image.open(path) as im:
        return np.asarray(im.convert('RGB'), dtype=np.uint8)


def prepare_data(data, device):
    """datasets.py:36-52."""
    rev_basic, rev_attrs, rev_mismatch_pair = data
    imgs, caps, cap_lens, cls_ids, keys = rev_basic
    real_imgs = [im.to(device) for im in imgs]
    caps = caps.squeeze().to(device)
    cap_lens = cap_lens.to(device)
    cls_ids = cls_ids.numpy()
    return [real_imgs, caps, cap_lens, cls_ids, keys]


class HostImageBatch(object):
    """A collated batch of HostImages as train.py's prepare_data consumes it
    (train.py:68-70: `len(imgs)` scales, `imgs[i].to(device)`): entry i is
    the batch at scale i; the first `.to(device)` of any scale runs the device
    transform for all of them (eegan_hip.pipeline), the others reuse it.
    Picklable, so DataLoader workers return it to the rank process."""

    def __init__(self, records, draws, imsize, base_size, branch_num, layout='nchw_f32'):
        self.records, self.draws = records, draws
        self.imsize, self.base_size, self.branch_num, self.layout = imsize, base_size, branch_num, layout
        self._outs = None

    def __getstate__(self):
        d = dict(self.__dict__)
        d['_outs'] = None
        return d

    def __len__(self):
        return self.branch_num

    def __getitem__(self, i):
        if not -self.branch_num <= i < self.branch_num:
            raise IndexError(i)
        return _ScaleImages(self, i % self.branch_num)

    def __iter__(self):
        return (self[i] for i in range(self.branch_num))

    def scale_shape(self, i):
        s = self.base_size * (2 ** i)
        return (len(self.records), 3, s, s)

    def tensors(self, device):
        device = torch.device(device)
        if self._outs is None or self._outs[0] != device:
            tf = _transform(device, self.imsize, self.base_size, self.branch_num, self.layout)
            outs, _ = tf(self.records, None, draws=self.draws)
            self._outs = (device, outs)
        return self._outs[1]


class _ScaleImages(object):
    """One scale of a HostImageBatch: `.to(device)` / `.cuda()` give the tensor."""

    def __init__(self, batch, i):
        self.batch, self.i = batch, i

    @property
    def shape(self):
        return torch.Size(self.batch.scale_shape(self.i))

    def size(self, dim=None):
        return self.shape if dim is None else self.shape[dim]

    def to(self, device, *args, **kwargs):
        return self.batch.tensors(device)[self.i]

    def cuda(self, device=None):
        return self.to('cuda' if device is None else device)


_TRANSFORMS = {}


def _transform(device, imsize, base_size, branch_num, layout):
    from eegan_hip.pipeline import DeviceImageTransform
    key = (str(device), imsize, base_size, branch_num, layout)
    if key not in _TRANSFORMS:
        _TRANSFORMS[key] = DeviceImageTransform(device, imsize=imsize, base_size=base_size,
                                                branch_num=branch_num, layout=layout)
    return _TRANSFORMS[key]


def collate_host_images(batch, *, collate_fn_map=None):
    """default_collate for a list of HostImages (registered below): the crop /
    flip draws of train.py's transform (train.py:269-272: Resize(304) ->
    RandomCrop(256) -> RandomHorizontalFlip) taken now, per sample in order,
    from torch's global generator of the collating process -- the generator
    the reference's transform draws from in its __getitem__."""
    from eegan_hip.pipeline import plan_draws
    sizes = batch[0].imsize or [cfg.TREE.BASE_SIZE * (2 ** i) for i in range(cfg.TREE.BRANCH_NUM)]
    if any(list(im.imsize or sizes) != list(sizes) for im in batch):
        raise ValueError('a batch mixes HostImages of different scale sets')
    base, branch, imsize = sizes[0], len(sizes), sizes[-1]
    records = [(im.rgb, im.bbox) for im in batch]
    return HostImageBatch(records, plan_draws(records, imsize, None), imsize, base, branch)


def _register_collate():
    from torch.utils.data._utils.collate import default_collate_fn_map
    default_collate_fn_map[HostImage] = collate_host_images


_register_collate()


class TextDataset(data.Dataset):
    """datasets.py:192-445 with the same constructor, loaders, getters and
    sample structure; `transform` is accepted for signature parity and must
    be None or the reference's train transform -- the image transform itself
    runs on the device when a batch's images are moved there.

    `shard=(rank, world)` (default: the process group's, see the module
    docstring) makes this rank's stride-`world` shard; the unpaired-caption
    draw still ranges over the whole split, as in the reference."""

    def __init__(self, data_dir, dataset_name, attr_name='EE-GAN', split='train', transform=None, shard=None):
        self.transform = transform
        self.split = split
        self.use_unpair = cfg.TRAIN.USE_UNPAIR
        self.use_attr = cfg.TRAIN.USE_ATTR
        base_size = cfg.TREE.BASE_SIZE
        branch_num = cfg.TREE.BRANCH_NUM
        self.imsize = [base_size * (2 ** i) for i in range(branch_num)]
        self.embedding_num = cfg.TEXT.CAPTIONS_PER_IMAGE
        self.data_dir = data_dir
        self.filenames = self.load_filenames(data_dir, split)
        self.captions, self.ixtoword, self.wordtoix, self.n_words = self.load_captions(data_dir, split)
        self.dataset_name = dataset_name
        self.bbox = self.load_bbox(data_dir) if dataset_name == 'bird' else None
        self.class_id = self.load_class_id(data_dir, split, len(self.filenames))
        self.number_example = len(self.filenames)
        if self.use_attr:
            self.attributes = self.load_attributes(data_dir, attr_name, split)
        self.iterator = self.prepare_train_pair
        if shard is None:
            from eegan_hip.launch import data_shard
            shard = data_shard()
        self.shard_rank, self.shard_world = int(shard[0]), int(shard[1])
        if not 0 <= self.shard_rank < self.shard_world:
            raise ValueError('shard %r: need 0 <= rank < world' % (shard,))
        if self.shard_world > 1:
            from eegan_hip.launch import offset_rank_rngs
            offset_rank_rngs(self.shard_rank)

    def base_index(self, index):
        """The split's sample behind this rank's item `index`."""
        if not 0 <= index < self.__len__():
            raise IndexError(index)
        return index * self.shard_world + self.shard_rank

    # --------------------------------------------------------- loaders --
    @staticmethod
    def load_filenames(data_dir, split):
        """datasets.py:231-239."""
        path = '%s/%s/filenames.pickle' % (data_dir, split)
        return load_pickle(path) if os.path.isfile(path) else []

    @staticmethod
    def load_bbox(data_dir):
        """datasets.py:242-246: {filename: [x, y, w, h]}."""
        return load_pickle(os.path.join(data_dir, 'bounding_boxes.pickle'))

    @staticmethod
    def load_attributes(data_dir, attr_name, split):
        """datasets.py:249-266: [train_attributes, test_attributes]."""
        x = load_pickle(os.path.join(data_dir, 'attributes/%s.pickle' % attr_name))
        return x[0] if split == 'train' else x[1]

    @staticmethod
    def load_captions(data_dir, split):
        """datasets.py:269-284: [train_captions, test_captions, ixtoword, wordtoix]."""
        x = load_pickle(os.path.join(data_dir, 'captions.pickle'))
        captions = x[0] if split == 'train' else x[1]
        return captions, x[2], x[3], len(x[2])

    @staticmethod
    def load_class_id(data_dir, split, total_num):
        """datasets.py:287-295 (python-2 pickles: bytes encoding)."""
        path = os.path.join(data_dir, split, 'class_info.pickle')
        if os.path.isfile(path):
            return load_pickle(path, encoding='bytes')
        return np.arange(total_num)

    # --------------------------------------------------------- getters --
    @staticmethod
    def get_attributes(sent_ix, attributes):
        """datasets.py:301-340 (same numpy.random draws)."""
        one = attributes[sent_ix]
        attr_num = len(one)
        out = np.zeros((cfg.TEXT.MAX_ATTR_NUM, cfg.TEXT.MAX_ATTR_LEN, 1), dtype='int64')
        rev_attr_num = min(cfg.TEXT.MAX_ATTR_NUM, attr_num)
        select_ixs = np.arange(rev_attr_num)
        np.random.shuffle(select_ixs)
        lens = np.ones((cfg.TEXT.MAX_ATTR_NUM, 1), dtype='int64')
        for cnt, ix in enumerate(select_ixs):
            attr = np.asarray(one[ix]).astype('int64')
            n = len(attr)
            if n == 0:
                continue
            if n <= cfg.TEXT.MAX_ATTR_LEN:
                out[cnt][:n, 0] = attr
                lens[cnt][0] = n
            else:
                ix = list(np.arange(n))
                np.random.shuffle(ix)
                ix = np.sort(ix[:cfg.TEXT.MAX_ATTR_LEN])
                out[cnt][:, 0] = attr[ix]
                lens[cnt][0] = cfg.TEXT.MAX_ATTR_LEN
        return out, rev_attr_num, lens

    @staticmethod
    def get_caption(sent_ix, captions):
        """datasets.py:342-361: zero-padded to WORDS_NUM, or a sorted random
        subset of WORDS_NUM words."""
        cap = np.asarray(captions[sent_ix]).astype('int64')
        if (cap == 0).sum() > 0:
            print('ERROR: do not need END (0) token', cap)
        n = len(cap)
        x = np.zeros((cfg.TEXT.WORDS_NUM, 1), dtype='int64')
        x_len = n
        if n <= cfg.TEXT.WORDS_NUM:
            x[:n, 0] = cap
        else:
            ix = list(np.arange(n))
            np.random.shuffle(ix)
            ix = np.sort(ix[:cfg.TEXT.WORDS_NUM])
            x[:, 0] = cap[ix]
            x_len = cfg.TEXT.WORDS_NUM
        return x, x_len

    def get_imgs(self, img_path, bbox=None):
        """datasets.py:391-424 up to the transform: decode, keep the bbox."""
        return HostImage(decode_rgb(img_path), None if bbox is None else [int(v) for v in bbox], list(self.imsize))

    def get_basic_pair(self, index):
        """datasets.py:363-374."""
        key = self.filenames[index]
        cls_id = self.class_id[index]
        bbox = self.bbox[key] if self.dataset_name == 'bird' else None
        image = self.get_imgs(os.path.join(self.data_dir, 'images', '%s.jpg' % key), bbox)
        cap, cap_len, sent_ix = self.get_cap_one(index)
        return image, cap, cap_len, cls_id, key, sent_ix

    def get_cap_unpair(self, cls_id):
        """datasets.py:376-382 (numpy randint: high exclusive), over the whole
        split (not this rank's shard)."""
        n = self.number_example
        unpair_idx = random.randint(0, n)
        while self.class_id[unpair_idx] == cls_id:
            unpair_idx = (unpair_idx + 1) % n
        caps, cap_len, _ = self.get_cap_one(unpair_idx)
        return caps, cap_len, self.class_id[unpair_idx], unpair_idx

    def get_cap_one(self, sent_index):
        """datasets.py:384-389."""
        sub_sent_ix = random.randint(0, self.embedding_num)
        sent_ix = sent_index * self.embedding_num + sub_sent_ix
        caps, cap_len = self.get_caption(sent_ix, self.captions)
        return caps, cap_len, sent_ix

    def prepare_train_pair(self, index):
        """datasets.py:426-439."""
        image, cap, cap_len, cls_id, key, sent_ix = self.get_basic_pair(index)
        ret_attrs = self.get_attributes(sent_ix, self.attributes) if self.use_attr else []
        if self.use_unpair:
            u_caps, u_len, u_cls, _ = self.get_cap_unpair(cls_id)
            ret_unpair = [u_caps, u_len, u_cls]
        else:
            ret_unpair = []
        return [image, cap, cap_len, cls_id, key], ret_attrs, ret_unpair

    def __len__(self):
        return len(self.filenames) // self.shard_world

    def __getitem__(self, index):
        return self.iterator(self.base_index(index))


class TextOnlyDataset(data.Dataset):
    """datasets.py:448-535, the sampling side's dataset (test.py:21, 122-128):
    captions (and attribute phrases) only, traversed per image (one random
    caption of each) or per sentence (`regard_sent`).  The reference calls
    TextDataset.load_class_id(data_dir, len(filenames)) without the split
    (datasets.py:465, a TypeError against its own signature at :287); here the
    split's class_info.pickle is loaded as the training set's is."""

    def __init__(self, data_dir, split='test', regard_sent=False, attr_name='EE-GAN'):
        self.embeddings_num = cfg.TEXT.CAPTIONS_PER_IMAGE
        self.split_name = split
        self.data_dir = data_dir
        self.regard_sent = regard_sent
        self.filenames = TextDataset.load_filenames(data_dir, split)
        self.captions, self.ixtoword, self.wordtoix, self.n_words = TextDataset.load_captions(data_dir, split)
        self.class_id = TextDataset.load_class_id(data_dir, split, len(self.filenames))
        self.get_caption = TextDataset.get_caption
        self.get_attributes = TextDataset.get_attributes
        if regard_sent:
            self.iterator = self.sent_regard_iter
            self.img_sum = self.__len__() // self.embeddings_num
        else:
            self.iterator = self.image_regard_iter
            self.img_sum = self.__len__()
        self.use_attr = cfg.TRAIN.USE_ATTR
        if self.use_attr:
            self.attributes = TextDataset.load_attributes(data_dir, attr_name, split)

    def image_regard_iter(self, img_ix):
        """datasets.py:482-488: a random caption of image img_ix."""
        caps, cap_len, sent_ix, _ = self.get_cap_one(img_ix)
        rev_attrs = self.get_attributes(sent_ix, self.attributes) if self.use_attr else []
        return [caps, cap_len, self.class_id[img_ix], self.filenames[img_ix]], rev_attrs

    def sent_regard_iter(self, sent_ix):
        """datasets.py:490-498."""
        caps, cap_len = self.get_caption(sent_ix, self.captions)
        img_ix = sent_ix // self.embeddings_num
        rev_attrs = self.get_attributes(sent_ix, self.attributes) if self.use_attr else []
        return [caps, cap_len, self.class_id[img_ix], self.filenames[img_ix]], rev_attrs

    def get_cap_one(self, img_index):
        """datasets.py:500-505 (numpy randint: high exclusive)."""
        sub_sent_ix = random.randint(0, self.embeddings_num)
        sent_ix = img_index * self.embeddings_num + sub_sent_ix
        caps, cap_len = self.get_caption(sent_ix, self.captions)
        return caps, cap_len, sent_ix, sub_sent_ix

    def __getitem__(self, index):
        return self.iterator(index)

    def __len__(self):
        return len(self.captions) if self.regard_sent else len(self.filenames)


def _collate(samples):
    """default_collate for everything but the images (kept as HostImage lists)."""
    from torch.utils.data import default_collate
    basic = [s[0] for s in samples]
    images = [b[0] for b in basic]
    rest = default_collate([b[1:] for b in basic])
    attrs = default_collate([s[1] for s in samples]) if samples[0][1] != [] else []
    unpair = default_collate([s[2] for s in samples]) if samples[0][2] != [] else []
    return [images] + list(rest), attrs, unpair


class DeviceDataLoader(object):
    """The reference's DataLoader (train.py:265-280) with the image transform
    on the GPU: host workers unpickle / draw captions / decode JPEGs, the main
    process runs eegan_hip.pipeline.DeviceImageTransform on each batch (crop /
    flip draws from `generator`, torchvision's order) and yields the
    reference's batch ([imgs, caps, cap_lens, cls_ids, keys], attrs, unpair)
    with imgs = three device tensors (64, 128, 256 px): NCHW fp32 as the
    reference's ('nchw_f32') or the drop-in models' NHWC bf16 ('nhwc_bf16')."""

    def __init__(self, dataset, batch_size, device, shuffle=True, drop_last=True, num_workers=None, seed=3407,
                 layout='nchw_f32'):
        from eegan_hip.pipeline import DeviceImageTransform
        if num_workers is None:
            num_workers = batch_size // 4    # train.py:276
        self.loader = data.DataLoader(dataset, batch_size=batch_size, drop_last=drop_last, shuffle=shuffle,
                                      num_workers=num_workers, collate_fn=_collate)
        imsize = dataset.imsize[-1]
        self.transform = DeviceImageTransform(device, imsize=imsize, base_size=dataset.imsize[0],
                                              branch_num=len(dataset.imsize), layout=layout)
        # a rank of a sharded dataset draws its own crops
        self.generator = torch.Generator().manual_seed(seed + getattr(dataset, 'shard_rank', 0))
        self.last_draws = None

    def __len__(self):
        return len(self.loader)

    def __iter__(self):
        for basic, attrs, unpair in self.loader:
            images = basic[0]
            imgs, self.last_draws = self.transform([(im.rgb, im.bbox) for im in images], self.generator)
            yield [imgs] + basic[1:], attrs, unpair
