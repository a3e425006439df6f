"""One rank of tests/test_launch_cpu.py (torchrun, CPU): importing the drop-in
package must join the ranks by itself (eegan_hip.launch) -- this script makes
no init call -- and the group must work (an all-reduce over gloo)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in (REPO, os.path.join(REPO, 'ee-gan_amd')):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402


def main(out):
    import miscc.config  # noqa: F401
    import models  # noqa: F401
    import torch.distributed as dist
    res = {'initialized': dist.is_initialized()}
    if res['initialized']:
        t = torch.tensor([float(dist.get_rank() + 1)])
        dist.all_reduce(t)
        res.update(world=dist.get_world_size(), rank=dist.get_rank(), sum=float(t))
    else:
        from eegan_hip.launch import check_process_group
        try:
            check_process_group()
            res['raised'] = False
        except RuntimeError as e:
            res['raised'] = True
            res['msg'] = str(e)
    torch.save(res, os.path.join(out, 'launch_rank%s.pt' % os.environ['RANK']))


if __name__ == '__main__':
    main(sys.argv[1])
