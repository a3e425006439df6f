"""Probe: host cost of submitting the captured step graph vs its GPU time.

Builds the bench workload (default C2), captures the step graph, then
  * steady state: wall time per replay over K back-to-back replays;
  * submission: the stream is first blocked by a ~0.3 s spin kernel, then ONE
    replay is submitted; the host time of that call is the pure submission
    cost (no queue back-pressure, the GPU cannot start it yet);
  * graph size: nodes / edges of the captured hipGraph (when torch exposes it).
Run once per runtime setting (env), e.g.
  python tools/probe/graph_submit.py --config C2
"""
import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, 'ee-gan_amd'))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def graph_size(g):
    try:
        raw = g.raw_cuda_graph()
    except Exception as e:  # noqa: BLE001
        return {'error': repr(e)[:120]}
    hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), 'lib', 'libamdhip64.so'))
    n = ctypes.c_size_t(0)
    rc = hip.hipGraphGetNodes(ctypes.c_void_p(raw), None, ctypes.byref(n))
    e = ctypes.c_size_t(0)
    rc2 = hip.hipGraphGetEdges(ctypes.c_void_p(raw), None, None, ctypes.byref(e))
    return {'nodes': n.value, 'edges': e.value, 'rc': [rc, rc2]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='C2')
    ap.add_argument('--steps', type=int, default=20)
    args = ap.parse_args()
    import bench
    from eegan_hip.trainer import StepGraph
    from eegan_hip.synthetic import make_batch
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    T, B, ncls = bench.build(args.config, dev)
    batch = make_batch(B, dev, seed=3407, class_num=ncls, with_class=True)
    torch.autograd.graph.set_warn_on_accumulate_grad_stream_mismatch(False)
    sg = StepGraph(T, batch, warmup=2, keep_graph=True)
    sg.replay()
    torch.cuda.synchronize()
    out = {'config': args.config, 'env': {k: v for k, v in os.environ.items()
                                          if k.startswith(('DEBUG_', 'GPU_', 'HIP_', 'AMD_', 'EEGAN_'))}}
    out['graph'] = graph_size(sg.graph)
    # steady state by replay depth (StepGraph.DEPTH: replays kept in flight, 0 = unpaced)
    paced = {}
    for rep in range(2):
        for depth in (0, 1, 2, 3):
            sg.DEPTH = depth
            sg._inflight = []
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                sg.replay()
            torch.cuda.synchronize()
            paced.setdefault(str(depth), []).append(round((time.perf_counter() - t0) / args.steps * 1e3, 3))
    out['ms_per_step_by_depth'] = paced
    sg.DEPTH = 0
    # steady state
    t0 = time.perf_counter()
    for _ in range(args.steps):
        sg.replay()
    t_issue = time.perf_counter() - t0
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    out['ms_per_step'] = dt / args.steps * 1e3
    out['host_issue_ms_per_step'] = t_issue / args.steps * 1e3
    out['img_s'] = B * args.steps / dt
    # pure submission: GPU blocked by a spin kernel on the replay stream
    subs = []
    for _ in range(3):
        torch.cuda.synchronize()
        torch.cuda._sleep(int(2.4e9 * 0.3))
        t0 = time.perf_counter()
        sg.replay()
        subs.append((time.perf_counter() - t0) * 1e3)
        torch.cuda.synchronize()
    out['submit_ms_blocked_gpu'] = subs
    # GPU time of one replay from an idle GPU, host submission included
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record()
    sg.replay()
    e1.record()
    torch.cuda.synchronize()
    out['single_replay_wall_ms'] = (time.perf_counter() - t0) * 1e3
    out['single_replay_event_ms'] = e0.elapsed_time(e1)
    print('GRAPHSUBMIT ' + json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
