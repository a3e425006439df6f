#!/bin/bash
# Kernel trace of the small-grid conv shapes (main kernel vs split-K reduce).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
S=${1:-c3x3_512_4,c3x3_256_8,c1x1_768_17}
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/convtrace -o run -- \
  python3 tools/conv_bench.py --iters 20 --shapes $S --dirs fwd,bwdd > gpurun_out/convtrace.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections
rows = []
for p in glob.glob('gpurun_out/convtrace/**/*kernel_trace.csv', recursive=True):
    rows += list(csv.DictReader(open(p)))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
agg = collections.OrderedDict()
prev_end = None
for r in rows:
    n = r['Kernel_Name'].replace('(anonymous namespace)::', '')[:60]
    key = (n, '%sx%sx%s' % (r.get('Grid_Size_X'), r.get('Grid_Size_Y'), r.get('Grid_Size_Z')), r.get('Workgroup_Size_X'))
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    gap = (int(r['Start_Timestamp']) - prev_end) / 1e3 if prev_end else 0
    prev_end = int(r['End_Timestamp'])
    a = agg.setdefault(key, [0, 0.0, 0.0, r.get('VGPR_Count', r.get('Arch_VGPR_Count')), r.get('LDS_Block_Size', r.get('Group_Segment_Size'))])
    a[0] += 1; a[1] += d; a[2] += gap
for (n, g, w), (c, t, gp, v, lds) in agg.items():
    print('%-60s grid %9s wg %4s vgpr %4s lds %6s  n %4d  avg %7.2f us  avg gap before %7.2f us' % (n, g, w, v, lds, c, t / c, gp / c))
PY
find gpurun_out/convtrace -name '*.csv' -delete
