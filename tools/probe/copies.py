"""Probe: where the step's device-to-device copies and fills come from (torch profiler, one eager step)."""
import os
import sys
import collections
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, 'ee-gan_amd'))
sys.path.insert(0, REPO)
import torch
from torch.profiler import profile, ProfilerActivity
import bench
from eegan_hip.synthetic import make_batch
dev = torch.device('cuda', 0)
T, B, ncls = bench.build('C2', dev)
T.use_streams = False
batch = make_batch(B, dev, class_num=max(ncls, 1))
T.train_step(batch)
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True, record_shapes=True) as prof:
    T.train_step(batch)
    torch.cuda.synchronize()
cnt = collections.Counter()
for ev in prof.events():
    if ev.device_type == torch.autograd.DeviceType.CPU and ev.name in ('aten::copy_', 'aten::fill_', 'aten::zero_',
                                                                       'aten::add', 'aten::add_', 'aten::mul',
                                                                       'aten::clone', 'aten::cat', 'aten::zeros'):
        st = [f for f in (ev.stack or []) if 'eegan' in f or 'models' in f or 'DAMSM' in f or 'trainer' in f]
        cnt[(ev.name, str(ev.input_shapes)[:50], ' < '.join(st[:2]))] += 1
for k, v in cnt.most_common(50):
    print(v, k)
names = collections.Counter(ev.name for ev in prof.events() if ev.device_type == torch.autograd.DeviceType.CUDA)
for k, v in names.most_common(15):
    print(v, k[:90])
