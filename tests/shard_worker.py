"""One rank of tests/test_data_shard_cpu.py's torchrun job: train.py's data
side, unchanged -- the drop-in modules imported first (train.py:22-29), the
'spawn' start method (train.py:35), the seeds (train.py:521-525), TextDataset +
DataLoader(shuffle=True, drop_last=True, workers) (train.py:274-278), the noise
draw (train.py:189).  No rank appears anywhere; the import joins the ranks
(eegan_hip.launch), the dataset shards itself and offsets ranks > 0's random
streams.  Also records a module's weights as initialised from those streams
and after eegan_hip.dist.broadcast_state (which the models run at their first
forward)."""
import multiprocessing
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in (REPO, os.path.join(REPO, 'ee-gan_amd')):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import miscc.config  # noqa: F401,E402
import sync_batchnorm  # noqa: F401,E402
from datasets import TextDataset  # noqa: E402
import models  # noqa: E402

multiprocessing.set_start_method('spawn', True)


def main(data_dir, out):
    random.seed(3407)
    np.random.seed(3407)
    torch.manual_seed(3407)
    ds = TextDataset(data_dir=data_dir, dataset_name='bird', transform=None)
    dl = torch.utils.data.DataLoader(ds, batch_size=3, drop_last=True, shuffle=True, num_workers=1)
    attr = models.ATTR_Enhance()
    flat = lambda m: torch.cat([p.detach().reshape(-1).clone() for p in m.parameters()])  # noqa: E731
    init = flat(attr)
    from eegan_hip import dist as D
    D.broadcast_state(attr)
    res = {'len': len(ds), 'epochs': [], 'draws': [], 'init': init, 'after': flat(attr)}
    for _ in range(2):
        keys = []
        for basic, attrs, unpair in dl:
            keys += list(basic[4])
            res['draws'].append(basic[0].draws)
        res['epochs'].append(keys)
    res['noise'] = torch.randn(3, 100)
    torch.save(res, os.path.join(out, 'shard_rank%s.pt' % os.environ['RANK']))


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
