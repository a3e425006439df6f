"""Probe: do independent branches of a captured HIP graph run concurrently?
Two (or one) streams each issue a chain of small kernels (few blocks each);
compare graph replay time of 1 stream x 2n kernels vs 2 streams x n."""
import torch
torch.cuda.set_device(0)
n = 200
xs = [torch.randn(64 * 1024, device='cuda') for _ in range(2)]


def chain(x, k):
    for _ in range(k):
        x.mul_(1.0001)   # one small elementwise kernel (64K elements)


def body(two):
    main = torch.cuda.current_stream()
    if not two:
        chain(xs[0], n)
        chain(xs[1], n)
        return
    s = [torch.cuda.Stream(), torch.cuda.Stream()]
    for st in s:
        st.wait_stream(main)
    for st, x in zip(s, xs):
        with torch.cuda.stream(st):
            chain(x, n)
    for st in s:
        main.wait_stream(st)


for two in (False, True):
    body(two)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body(two)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    print('streams=%d  %.1f us per replay (%d kernels)' % (2 if two else 1, e0.elapsed_time(e1) * 100, 2 * n),
          flush=True)

# two separately captured graphs, replayed on two streams concurrently
gs = []
ss = [torch.cuda.Stream(), torch.cuda.Stream()]
for x, st in zip(xs, ss):
    g = torch.cuda.CUDAGraph()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        chain(x, n)
        with torch.cuda.graph(g, stream=st):
            chain(x, n)
    torch.cuda.current_stream().wait_stream(st)
    gs.append(g)
torch.cuda.synchronize()


def replay_two():
    main = torch.cuda.current_stream()
    for st in ss:
        st.wait_stream(main)
    for g, st in zip(gs, ss):
        with torch.cuda.stream(st):
            g.replay()
    for st in ss:
        main.wait_stream(st)


for _ in range(3):
    replay_two()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10):
    replay_two()
e1.record()
torch.cuda.synchronize()
print('2 graphs on 2 streams  %.1f us per replay pair (%d kernels)' % (e0.elapsed_time(e1) * 100, 2 * n), flush=True)
