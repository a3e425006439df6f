"""Probe: own RCCL communicator (eegan_hip.rccl) eager and under HIP-graph capture, one rank.
    python rccl_probe.py CASE   (simple | streams | many | fp64 | gather | global)"""
import os
import sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, 'ee-gan_amd'))
import torch
torch.cuda.set_device(0)
from eegan_hip import dist as D
case = sys.argv[1] if len(sys.argv) > 1 else 'simple'
D.init_from_env()
t = torch.ones(1 << 20, device='cuda')
u = torch.ones(64, dtype=torch.float64, device='cuda')
side = [torch.cuda.Stream() for _ in range(3)]


def body():
    if case == 'simple' or case == 'global':
        t.mul_(2)
        D.all_reduce(t)
    elif case == 'streams':
        main = torch.cuda.current_stream()
        for s in side:
            s.wait_stream(main)
        for s in side:
            with torch.cuda.stream(s):
                x = torch.ones(4096, device='cuda')
                D.all_reduce(x)
                t.add_(x[0])
        for s in side:
            main.wait_stream(s)
    elif case == 'many':
        for _ in range(60):
            D.all_reduce(t[:1000])
    elif case == 'fp64':
        for _ in range(10):
            D.all_reduce(u)
    elif case == 'gather':
        g = D._gather(t[:600].view(2, 300))
        t[:10].add_(g[0, :10])


s0 = torch.cuda.Stream()
s0.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s0):
    body()
torch.cuda.current_stream().wait_stream(s0)
torch.cuda.synchronize()
print(case, 'eager ok', flush=True)
graph = torch.cuda.CUDAGraph()
with torch.cuda.graph(graph, capture_error_mode='global' if case == 'global' else 'thread_local'):
    body()
print(case, 'captured', flush=True)
graph.replay()
torch.cuda.synchronize()
print(case, 'replay ok', flush=True)
