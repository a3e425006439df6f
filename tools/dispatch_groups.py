"""Group the dispatches of a rocprofv3 kernel trace by (kernel, grid) and
list the groups that take the most time per step, so the shapes worth
tuning can be read off a graph-replayed bench run.

    python tools/dispatch_groups.py TRACE_DIR --steps N [--filter conv] [--top 40]

--steps 0: steps counted from the trace (adam_tick_kernel dispatches / --ticks,
one tick per optimizer step: 7 per C2 train step -- G and each D twice).
"""
import argparse
import csv
import glob
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('trace')
    ap.add_argument('--steps', type=int, required=True)
    ap.add_argument('--ticks', type=int, default=7, help='adam_tick_kernel dispatches per train step')
    ap.add_argument('--filter', default='')
    ap.add_argument('--top', type=int, default=40)
    ap.add_argument('--by-name', action='store_true', help='group by kernel name only, sort by calls')
    args = ap.parse_args()
    groups = defaultdict(lambda: [0, 0])
    ticks = 0
    for path in glob.glob(os.path.join(args.trace, '**', '*kernel_trace.csv'), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                name = r['Kernel_Name']
                ticks += 'adam_tick_kernel' in name
                if args.filter and args.filter not in name:
                    continue
                short = name.replace('(anonymous namespace)::', '').replace('void ', '')
                short = short.split('(')[0][:90]
                grid = (r.get('Grid_Size_X', r.get('Grid_Size', '?')), r.get('Grid_Size_Y', ''),
                        r.get('Grid_Size_Z', ''))
                g = groups[(short, ('',) if args.by_name else grid)]
                g[0] += 1
                g[1] += int(r['End_Timestamp']) - int(r['Start_Timestamp'])
    if args.steps <= 0:
        args.steps = max(1, round(ticks / args.ticks))
        print('steps: %d (%d adam ticks / %d)' % (args.steps, ticks, args.ticks))
    rows = sorted(groups.items(), key=lambda kv: -kv[1][0 if args.by_name else 1])
    tot = sum(v[1] for v in groups.values())
    print('total %.3f ms/step over %d groups' % (tot * 1e-6 / args.steps, len(groups)))
    for (k, grid), (n, ns) in rows[:args.top]:
        print('%7.3f ms/step %5.1f calls/step %8.2f us  grid %-20s %s' % (
            ns * 1e-6 / args.steps, n / args.steps, ns * 1e-3 / n, 'x'.join(x for x in grid if x), k))


if __name__ == '__main__':
    main()
