#!/usr/bin/env python
"""Throughput of the device input transform (eegan_hip.pipeline) against the
reference's per-image PIL chain (oracle/pipeline_oracle.get_imgs, one core):
CUB-like decoded images (500 x 375 .. 500 x 500, bbox crops), batch B.

    python tools/pipeline_bench.py [--batch 16] [--iters 20]

Prints one JSON line: GPU images/s with the host planning + H2D copy
(`end_to_end`) and the GPU kernels alone (`kernels`, HIP events), and the CPU
PIL chain images/s on one thread.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'ee-gan_amd'))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=16)
    ap.add_argument('--iters', type=int, default=20)
    args = ap.parse_args()
    from eegan_hip.pipeline import DeviceImageTransform
    from oracle import pipeline_oracle as PO
    dev = torch.device('cuda', 0)
    rs = np.random.RandomState(0)
    recs = []
    for b in range(args.batch):
        w, h = 500, int(rs.randint(375, 501))
        bw, bh = int(rs.randint(200, w)), int(rs.randint(150, h))
        recs.append((rs.randint(0, 256, size=(h, w, 3)).astype(np.uint8),
                     [int(rs.randint(0, w - bw + 1)), int(rs.randint(0, h - bh + 1)), bw, bh]))
    tf = DeviceImageTransform(dev, layout='nhwc_bf16')
    g = torch.Generator().manual_seed(1)
    for _ in range(3):
        tf(recs, g)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.iters):
        tf(recs, g)
    torch.cuda.synchronize()
    e2e = args.batch * args.iters / (time.perf_counter() - t0)
    # kernels alone: the host plan and the upload done once, the launch timed with events
    from eegan_hip import pipeline as P
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    orig = P.ops.pipe_transform
    times = []

    def timed(*a):
        e0.record()
        orig(*a)
        e1.record()
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1))
    P.ops.pipe_transform = timed
    try:
        for _ in range(args.iters):
            tf(recs, g)
    finally:
        P.ops.pipe_transform = orig
    k_ms = sorted(times)[len(times) // 2]
    torch.set_num_threads(1)
    gc = torch.Generator().manual_seed(1)
    n_cpu = min(args.batch, 8)
    t0 = time.perf_counter()
    for rgb, bbox in recs[:n_cpu]:
        PO.get_imgs(rgb, bbox, generator=gc)
    cpu = n_cpu / (time.perf_counter() - t0)
    print(json.dumps({'batch': args.batch, 'gpu_end_to_end_img_s': round(e2e, 1),
                      'gpu_kernels_ms_per_batch': round(k_ms, 4),
                      'gpu_kernels_img_s': round(args.batch / k_ms * 1e3, 1),
                      'cpu_pil_img_s_1thread': round(cpu, 1),
                      'note': 'end_to_end includes the host weight planning and the pinned H2D copy of the '
                              'decoded sub-rectangles; JPEG decoding excluded on both sides'}), flush=True)


if __name__ == '__main__':
    main()
