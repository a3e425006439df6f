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
GRBM_GUI_ACTIVE` run: MFMA-busy SIMD cycles per call (summed over the
1024 SIMDs; a 16x16x32 bf16 MFMA is 16 busy cycles for 16384 FLOP, 1024
FLOP per busy cycle per SIMD -- MI355X_MICROARCH.md, matrix cores).
mfma_util = busy cycles / (the call's duration in the kernel-trace pass x
2.4 GHz x 1024 SIMDs): the fraction of the dense bf16 MFMA peak, on the
same time base as bench.py's FLOP-derived fraction (which it can only exceed
by the MFMAs spent on padding).  GRBM_GUI_ACTIVE (summed over the 8 XCDs)
is kept as gpu_active_cycles_per_call for reference only: on dispatches
shorter than ~0.3 ms it reads well above duration x clock (MI355X_MICROARCH.md,
DVFS give-back), so it is not used as the denominator.
The summary records the git commit and the sha256 of libeegan_hip.so it was
taken with, so bench.py can flag a summary taken with other kernels.
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
    (re.compile(r'conv_halo3_kernel<0,'), 'conv_fwd', True),
    (re.compile(r'conv_halo3_kernel<1,'), 'conv_bwd_data', True),
    (re.compile(r'colsum_rows_kernel<.*WgradMap'), 'conv_bwd_weight', False),
]


CLOCK_HZ = 2.4e9   # MI355X max clock (MI355X_MICROARCH.md): a lower bound on the busy fraction under DVFS
SIMDS = 1024


def _provenance():
    import hashlib
    import subprocess
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    so = os.path.join(repo, 'ee-gan_amd', 'eegan_hip', 'libeegan_hip.so')
    h = hashlib.sha256()
    try:
        with open(so, 'rb') as f:
            h.update(f.read())
        sha = h.hexdigest()[:16]
    except OSError:
        sha = None
    try:
        head = subprocess.run(['git', 'rev-parse', '--short=12', 'HEAD'], cwd=repo, capture_output=True,
                              text=True).stdout.strip() or None
    except OSError:
        head = None
    head = head or os.environ.get('EEGAN_GIT_HEAD')   # the GPU box's copy of the tree has no .git
    return {'lib_sha256_16': sha, 'git_head': head}


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
    ap.add_argument('--config', default='C2', help='bench.py workload the runs were taken on')
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
        if busy and busy[0].get(fam):
            b = busy[0][fam]
            n = max(busy[1][fam], 1)
            e['mfma_busy_cycles_per_call'] = round(b / n)
            e['mfma_util'] = round(b / n / (e['avg_call_us'] * 1e-6 * CLOCK_HZ * SIMDS), 4)
            e['mfma_util_unit'] = ('SQ_VALU_MFMA_BUSY_CYCLES per call / (kernel-trace call duration x 2.4 GHz x '
                                   '1024 SIMDs)')
            if gui and gui[0].get(fam):
                e['gpu_active_cycles_per_call'] = round(gui[0][fam] / 8 / n)
        out[fam] = e
    total_ns = sum(o['ns'] for o in fams.values())
    res = {'families': out, 'gpu_busy_ms_total': round(total_ns * 1e-6, 3), 'config': a.config}
    res.update(_provenance())
    if a.steps <= 0:   # counted: one adam_tick_kernel per optimizer step, 7 per C2 train step
        ticks = fams.get('adam_tick_kernel', {}).get('calls', 0)
        a.steps = round(ticks / 7) if ticks else 0
    if a.steps:
        res['steps'] = a.steps
        res['gpu_busy_ms_per_step'] = round(total_ns * 1e-6 / a.steps, 3)
        for e in out.values():
            e['ms_per_step'] = round(e['total_ms'] / a.steps, 3)
    txt = json.dumps(res, indent=1)
    if a.out:
        with open(a.out, 'w') as f:
            f.write(txt + '\n')
    print(txt)


if __name__ == '__main__':
    main()
