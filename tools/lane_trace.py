#!/usr/bin/env python
"""Kernel-level breakdown of one discriminator's d_update (train.py:437-469)
by phase: run `Trainer._d_update_one(i, ...)` eagerly on one stream with
phase stamps on (Fn.stamp: stamp_kernel dispatches mark the boundaries), under
rocprofv3 --kernel-trace; then `--report DIR` groups the trace's kernels by
phase and by kernel, so the lane's time can be read per kernel.

    rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python3 tools/lane_trace.py --d 2
    python3 tools/lane_trace.py --report OUT
"""
import argparse
import collections
import csv
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'ee-gan_amd'))
sys.path.insert(0, REPO)
PHASES = os.path.join(REPO, 'gpurun_out', 'lane_phases.json')


def run(args):
    import torch
    import bench
    from eegan_hip import functional as Fn
    from eegan_hip.synthetic import make_batch
    dev = torch.device('cuda', 0)
    T, B, ncls = bench.build(args.config, dev)
    T.use_streams = False
    batch = make_batch(B, dev, class_num=ncls, with_class=True)
    T.train_step(batch)
    words, sent, attrs, unpair = T.encode_text(batch)
    class_labels = Fn.class_onehot(batch['cls_ids'], B, ncls, dev)[0] if T.disc_class else None
    with torch.no_grad():
        _, att = T.attr_enhance(sent, attrs)
        fakes = T.netG(torch.randn(B, 100, device=dev), sent, T.attr_enhance.module.attr_merge(att))
    fakes = [f.detach() for f in fakes]
    if args.d >= 0:
        for _ in T._d_update_one(args.d, batch['imgs'], fakes, sent, unpair, class_labels, False):
            pass
    torch.cuda.synchronize()
    Fn.STAMP_BUF = torch.zeros(4096, dtype=torch.int64, device=dev)
    names = []
    for _ in range(args.reps):
        Fn.STAMPS = []
        if args.d < 0:   # the whole step, one stream
            T.train_step(batch)
        else:
            Fn.stamp('start')
            for _ in T._d_update_one(args.d, batch['imgs'], fakes, sent, unpair, class_labels, False):
                pass
        names = [n for n, _ in Fn.STAMPS]
        Fn.STAMPS = None
    torch.cuda.synchronize()
    os.makedirs(os.path.dirname(PHASES), exist_ok=True)
    with open(PHASES, 'w') as f:
        json.dump({'names': names, 'reps': args.reps}, f)


TOP = int(os.environ.get("LANE_TOP", "14"))


def report(d):
    meta = json.load(open(PHASES))
    names, reps = meta['names'], meta['reps']
    rows = []
    for p in glob.glob(os.path.join(d, '**', '*kernel_trace.csv'), recursive=True):
        rows += list(csv.DictReader(open(p)))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    # the last reps x len(names) stamps delimit the stamped repetitions
    idx = [k for k, r in enumerate(rows) if 'stamp_kernel' in r['Kernel_Name']]
    idx = idx[-reps * len(names):]
    per = collections.defaultdict(lambda: collections.defaultdict(lambda: [0, 0]))
    span = collections.defaultdict(float)
    for rep in range(reps):
        for j in range(1, len(names)):
            a, b = idx[rep * len(names) + j - 1], idx[rep * len(names) + j]
            span[names[j]] += (int(rows[b]['Start_Timestamp']) - int(rows[a]['End_Timestamp'])) / 1e3 / reps
            for r in rows[a + 1:b]:
                k = r['Kernel_Name'].replace('(anonymous namespace)::', '').replace('void ', '').split('(')[0][:60]
                g = '%sx%sx%s' % (r.get('Grid_Size_X'), r.get('Grid_Size_Y'), r.get('Grid_Size_Z'))
                e = per[names[j]][(k, g)]
                e[0] += 1
                e[1] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    for ph in names[1:]:
        tot = sum(v[1] for v in per[ph].values()) / reps
        n = sum(v[0] for v in per[ph].values()) / reps
        print('== %s: span %.1f us, kernels %.0f, kernel time %.1f us' % (ph, span[ph], n, tot))
        for (k, g), (c, t) in sorted(per[ph].items(), key=lambda kv: -kv[1][1])[:TOP]:
            print('   %8.1f us %4.0f x  %-60s %s' % (t / reps, c / reps, k, g))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='C2')
    ap.add_argument('--d', type=int, default=2, help='discriminator index; -1: the whole step')
    ap.add_argument('--reps', type=int, default=3)
    ap.add_argument('--report')
    args = ap.parse_args()
    if args.report:
        report(args.report)
    else:
        run(args)


if __name__ == '__main__':
    main()
