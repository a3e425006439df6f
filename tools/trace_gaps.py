"""Busy time vs wall span of a rocprofv3 kernel trace (graph replay gaps).

    python tools/trace_gaps.py TRACE_DIR [--last N]   (N = kernels of the last N dispatch groups)
"""
import csv
import glob
import os
import sys
from collections import Counter

d = sys.argv[1]
rows = []
for path in glob.glob(os.path.join(d, '**', '*kernel_trace.csv'), recursive=True):
    with open(path) as f:
        rows += list(csv.DictReader(f))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
t = [(int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']) for r in rows]
n = len(t)
# take the middle half of the trace (steady replays)
a, b = n // 4, 3 * n // 4
seg = t[a:b]
busy = sum(e - s for s, e, _ in seg)
span = max(e for _, e, _ in seg) - seg[0][0]
# union of the kernel intervals (concurrent streams overlap)
cov, cur_s, cur_e = 0, None, None
for s_, e_, _ in seg:
    if cur_e is None or s_ > cur_e:
        if cur_e is not None:
            cov += cur_e - cur_s
        cur_s, cur_e = s_, e_
    else:
        cur_e = max(cur_e, e_)
cov += cur_e - cur_s
print('union busy %.2f ms of span %.2f ms (idle %.2f ms)' % (cov * 1e-6, span * 1e-6, (span - cov) * 1e-6))
gaps = [seg[i + 1][0] - seg[i][1] for i in range(len(seg) - 1)]
gaps.sort()
print('kernels %d  busy %.2f ms  span %.2f ms  busy/span %.3f' % (len(seg), busy * 1e-6, span * 1e-6, busy / span))
print('gap median %.2f us  p90 %.2f us  total %.2f ms' % (gaps[len(gaps) // 2] * 1e-3, gaps[int(len(gaps) * .9)] * 1e-3,
                                                            sum(g for g in gaps if g > 0) * 1e-6))
def short(k):
    return k.replace('(anonymous namespace)::', '').replace('void ', '').split('(')[0][:60]


c = Counter()
tm = Counter()
for s_, e_, k in seg:
    c[short(k)] += 1
    tm[short(k)] += e_ - s_
for k, v in tm.most_common(25):
    print('%6d %8.2f ms  %s' % (c[k], v * 1e-6, k))
