#!/bin/bash
# Kernel trace of the DAMSM microbench (per-kernel average durations).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/dtrace -o run -- \
  python3 tools/damsm_bench.py --reps 10 > gpurun_out/dtrace.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections
rows = []
for p in glob.glob('gpurun_out/dtrace/**/*kernel_trace.csv', recursive=True):
    rows += list(csv.DictReader(open(p)))
agg = collections.OrderedDict()
for r in sorted(rows, key=lambda r: int(r['Start_Timestamp'])):
    n = r['Kernel_Name'].replace('(anonymous namespace)::', '')[:50]
    key = (n, '%sx%sx%s' % (r.get('Grid_Size_X'), r.get('Grid_Size_Y'), r.get('Grid_Size_Z')))
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    a = agg.setdefault(key, [0, 0.0, r.get('Arch_VGPR_Count', r.get('VGPR_Count')), r.get('Group_Segment_Size', r.get('LDS_Block_Size'))])
    a[0] += 1; a[1] += d
for (n, g), (c, t, v, l) in agg.items():
    if 'damsm' in n or 'words' in n or c >= 10:
        print('%-50s grid %-16s vgpr %4s lds %6s  n %4d  avg %8.2f us' % (n, g, v, l, c, t / c))
PY
find gpurun_out/dtrace -name '*.csv' -delete
