"""Probe: fork/join of one shared 'communication' stream from several side
streams inside a HIP-graph capture (the pattern eegan_hip.rccl uses).
    python stream_probe.py CASE  (work | empty | nojoin_comm)"""
import sys
import torch
torch.cuda.set_device(0)
case = sys.argv[1]
t = torch.ones(1 << 20, device='cuda')
side = [torch.cuda.Stream() for _ in range(3)]
comm = torch.cuda.Stream()


def coll(x):
    cur = torch.cuda.current_stream()
    comm.wait_stream(cur)
    with torch.cuda.stream(comm):
        if case != 'empty':
            x.mul_(1.0)
    cur.wait_stream(comm)


def body():
    main = torch.cuda.current_stream()
    for s in side:
        s.wait_stream(main)
    for s in side:
        with torch.cuda.stream(s):
            x = torch.ones(4096, device='cuda')
            coll(x)
            t.add_(x[0])
    for s in side:
        main.wait_stream(s)
    if case == 'nojoin_comm':
        pass


s0 = torch.cuda.Stream()
s0.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s0):
    body()
torch.cuda.current_stream().wait_stream(s0)
torch.cuda.synchronize()
print(case, 'eager ok', flush=True)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, capture_error_mode='thread_local'):
    body()
print(case, 'captured', flush=True)
g.replay()
torch.cuda.synchronize()
print(case, 'replay ok', t[0].item(), flush=True)
