#!/usr/bin/env python
"""Summarise rocprofv3 output of a bench.py run per kernel family.

    python tools/rocprof_families.py --trace DIR [--fetch DIR] [--write DIR] [--steps K] [--out FILE]

--trace: directory of a `rocprofv3 --kernel-trace --stats` run; the kernel
trace gives, for each family, the dispatch count and the average duration of
one *call* (a conv call is the implicit-GEMM kernel plus, when split-K is
used, its reduce kernel -- the same bracket bench.py's HIP events time).
--fetch/--write: directories of separate `rocprofv3 --pmc FETCH_SIZE` /
`--pmc WRITE_SIZE` runs of the same command.  Per the MI355X guide (HBM
section) FETCH_SIZE on gfx950 counts half the bytes of wide coalesced reads,
so it is doubled; WRITE_SIZE is taken as is.  Both are in KB.
--mfma: directory of a `rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES
GRBM_GUI_ACTIVE` run: MFMA-busy SIMD cycles and GPU-active cycles (summed
over the 8 XCDs, so /8 per XCD) per call; mfma_util = busy / (active/8 x 1024
SIMDs), the fraction of the dense bf16 MFMA peak at the clock the kernel ran
(a 16x16x32 bf16 MFMA is 16 busy cycles for 16384 FLOP: 1024 FLOP per busy
cycle per SIMD -- MI355X_MICROARCH.md, matrix cores).
Output JSON: {family: {calls, avg_call_us, total_ms, hbm_bytes_per_call,
mfma_util}} plus totals (GPU busy time per step), read by bench.py for
`traffic` and `mfma_busy`.
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict

# (family, is_primary): the primary kernel counts calls; secondaries add time
_FAMILIES = [
    (re.compile(r'conv_fast_kernel<0,'), 'conv_fwd', True),
    (re.compile(r'conv_fast_kernel<1,'), 'conv_bwd_data', True),
    (re.compile(r'conv_wgrad_fast_kernel<'), 'conv_bwd_weight', True),
    (re.compile(r'conv_glds_kernel<0,'), 'conv_fwd', True),
    (re.compile(r'conv_glds_kernel<1,'), 'conv_bwd_data', True),
    (re.compile(r'conv_wgrad_glds_kernel<'), 'conv_bwd_weight', True),
    (re.compile(r'conv_igemm_kernel<0,'), 'conv_fwd', True),
    (re.compile(r'conv_splitk_reduce_kernel<0>'), 'conv_fwd', False),
    (re.compile(r'conv_igemm_kernel<1,'), 'conv_bwd_data', True),
    (re.compile(r'conv_splitk_reduce_kernel<1>'), 'conv_bwd_data', False),
    (re.compile(r'conv_wgrad_kernel<'), 'conv_bwd_weight', True),
    (re.compile(r'conv_thin(_lds)?_kernel<0,'), 'conv_fwd', True),
    (re.compile(r'conv_thin(_lds)?_kernel<1,'), 'conv_bwd_data', True),
    (re.compile(r'conv_wgrad_thin_kernel<'), 'conv_bwd_weight', True),
    (re.compile(r'conv_1x1_kernel<0,'), 'conv_fwd', True),
    (re.compile(r'conv_1x1_kernel<1,'), 'conv_bwd_data', True),
    (re.compile(r'conv_s2bwd_lds_kernel<'), 'conv_bwd_data', True),
    (re.compile(r'colsum_rows_kernel<.*WgradMap'), 'conv_bwd_weight', False),
]


def family(name):
    for rx, fam, prim in _FAMILIES:
        if rx.search(name):
            return fam, prim
    base = name.replace('(anonymous namespace)::', '').replace('void ', '')
    return re.sub(r'[<(].*', '', base).strip(), True


def _find(d, suffix):
    hits = sorted(glob.glob(os.path.join(d, '**', '*' + suffix), recursive=True))
    if not hits:
        raise FileNotFoundError('no *%s under %s' % (suffix, d))
    return hits


def kernel_trace(d):
    fams = defaultdict(lambda: {'calls': 0, 'dispatches': 0, 'ns': 0})
    for path in _find(d, 'kernel_trace.csv'):
        with open(path) as f:
            for row in csv.DictReader(f):
                fam, prim = family(row['Kernel_Name'])
                o = fams[fam]
                o['dispatches'] += 1
                o['calls'] += int(prim)
                o['ns'] += int(row['End_Timestamp']) - int(row['Start_Timestamp'])
    return fams


def pmc(d, counter):
    tot = defaultdict(float)
    calls = defaultdict(int)
    for path in _find(d, 'counter_collection.csv'):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row['Counter_Name'] != counter:
                    continue
                fam, prim = family(row['Kernel_Name'])
                tot[fam] += float(row['Counter_Value'])
                calls[fam] += int(prim)
    return tot, calls


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--trace', required=True)
    ap.add_argument('--fetch')
    ap.add_argument('--write')
    ap.add_argument('--mfma')
    ap.add_argument('--steps', type=int, default=0, help='steps in the traced run (warmup+timed) for per-step totals')
    ap.add_argument('--out')
    a = ap.parse_args()
    fams = kernel_trace(a.trace)
    fetch = pmc(a.fetch, 'FETCH_SIZE') if a.fetch else None
    write = pmc(a.write, 'WRITE_SIZE') if a.write else None
    busy = pmc(a.mfma, 'SQ_VALU_MFMA_BUSY_CYCLES') if a.mfma else None
    gui = pmc(a.mfma, 'GRBM_GUI_ACTIVE') if a.mfma else None
    out = {}
    for fam, o in sorted(fams.items(), key=lambda kv: -kv[1]['ns']):
        calls = max(o['calls'], 1)
        e = {'calls': o['calls'], 'dispatches': o['dispatches'], 'total_ms': round(o['ns'] * 1e-6, 3),
             'avg_call_us': round(o['ns'] / calls * 1e-3, 2)}
        if fetch and write and fam in fetch[0] and fam in write[0]:
            # KB -> bytes; FETCH_SIZE x2 (gfx950 wide-read correction)
            rd = 2.0 * fetch[0][fam] * 1024 / max(fetch[1][fam], 1)
            wr = write[0][fam] * 1024 / max(write[1][fam], 1)
            e['hbm_read_bytes_per_call'] = round(rd)
            e['hbm_write_bytes_per_call'] = round(wr)
            e['hbm_bytes_per_call'] = round(rd + wr)
        if busy and gui and gui[0].get(fam):
            b, gcy = busy[0][fam], gui[0][fam]
            n = max(busy[1][fam], 1)
            e['mfma_busy_cycles_per_call'] = round(b / n)
            e['gpu_active_cycles_per_call'] = round(gcy / 8 / n)
            e['mfma_util'] = round(b / (gcy / 8 * 1024), 4)
        out[fam] = e
    total_ns = sum(o['ns'] for o in fams.values())
    res = {'families': out, 'gpu_busy_ms_total': round(total_ns * 1e-6, 3)}
    if a.steps:
        res['gpu_busy_ms_per_step'] = round(total_ns * 1e-6 / a.steps, 3)
    txt = json.dumps(res, indent=1)
    if a.out:
        with open(a.out, 'w') as f:
            f.write(txt + '\n')
    print(txt)


if __name__ == '__main__':
    main()
