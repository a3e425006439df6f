"""Kernel time per step by kernel name (template arguments dropped) from a
rocprofv3 --stats kernel_stats.csv: python3 tools/kernel_families.py CSV STEPS [TOP]."""
import collections
import csv
import re
import sys


def main(path, steps, top=60):
    agg, calls = collections.Counter(), collections.Counter()
    for r in csv.DictReader(open(path)):
        n = r['Name'].replace('(anonymous namespace)::', '').replace('void ', '')
        if 'spin_kernel' in n:
            continue
        n = re.sub(r'[<(].*$', '', n).strip()
        agg[n] += float(r['TotalDurationNs']) / 1e6 / steps
        calls[n] += int(r['Calls']) / steps
    print('total kernel time %.3f ms/step' % sum(agg.values()))
    for k, v in agg.most_common(top):
        print('%8.3f ms %7.1f calls  %s' % (v, calls[k], k[:90]))


if __name__ == '__main__':
    main(sys.argv[1], float(sys.argv[2]), int(sys.argv[3]) if len(sys.argv) > 3 else 60)
