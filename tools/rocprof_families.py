#!/usr/bin/env python
"""Summarise rocprofv3 output of a bench.py run per kernel family.

    python tools/rocprof_families.py --trace DIR [--fetch DIR] [--write DIR] [--mfma DIR]
                                     [--bench-line LOG] [--steps K] [--out FILE]

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

Windows: bench.py launches a marker kernel (stamp_kernel) at both ends of its
timed region (the graph replays) and of its eager timing pass; the families
are summed over the timed replays only (in-step durations, lanes running
concurrently), `timing_pass` over the timing pass (single stream, what the
line's HIP events time).  --bench-line adds each conv family's algorithmic
FLOPs / bytes per call from the same run's line, and from them `frac_in_step`
(algorithmic FLOPs per step / in-step kernel time / 2.5 PFLOP/s),
`pmc_over_algorithmic` and the conv path's algorithmic and PMC HBM fractions
-- the figures bench.py then quotes, recomputable from this file alone.
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

# ONE kernel -> family table for every conv kernel in csrc/conv.hip, the same op
# families bench.py's event timer uses (functional.conv_fwd_raw / conv_bwd_data_raw /
# conv_bwd_weight_raw time every dispatch of one call: the GEMM kernel -- whichever
# specialised form the planner picked -- and, with split-K, its reduce).  (regex,
# family, is_primary): a primary kernel counts a call; secondaries add time and
# bytes to the call.  Ordered: the first match wins (conv_s2bwd_lds_kernel<NT, NC>
# and conv_wgrad_*<...> carry no mode argument, so they precede the mode rules).
# An unclassified kernel whose name starts with conv_ is an error (check_complete).
_FAMILIES = [
    (re.compile(r'conv_splitk_reduce_kernel<0>'), 'conv_fwd', False),
    (re.compile(r'conv_splitk_reduce_kernel<1>'), 'conv_bwd_data', False),
    (re.compile(r'conv_s2fwd_kernel'), 'conv_fwd', True),
    (re.compile(r'conv_s2bwd_lds_kernel<'), 'conv_bwd_data', True),
    (re.compile(r'conv_wgrad_\w*kernel<'), 'conv_bwd_weight', True),
    (re.compile(r'wgrad_quad_reduce_kernel<'), 'conv_bwd_weight', False),
    (re.compile(r'colsum_rows_kernel<.*WgradMap'), 'conv_bwd_weight', False),
    (re.compile(r'conv_(fast|glds|igemm|thin|thin_lds|1x1|halo3|halo3r)_kernel<0[,>]'), 'conv_fwd', True),
    (re.compile(r'conv_(fast|glds|igemm|thin|thin_lds|1x1|halo3|halo3r)_kernel<1[,>]'), 'conv_bwd_data', True),
]
CONV_FAMILIES = ('conv_fwd', 'conv_bwd_data', 'conv_bwd_weight')
MARKER = 'stamp_kernel'   # bench.py's window markers (eegan_stamp): timed region, then the timing pass
MFMA_PEAK = 2.5e15        # dense bf16 FLOP/s (MI355X_MICROARCH.md)
HBM_PEAK = 8.0e12         # B/s


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


def _short(name):
    return name.replace('(anonymous namespace)::', '').replace('void ', '').strip()


def family(name):
    for rx, fam, prim in _FAMILIES:
        if rx.search(name):
            return fam, prim
    return re.sub(r'[<(].*', '', _short(name)).strip(), True


def check_complete(names):
    """Every conv kernel of the run must be in the table (else the families
    silently lose time and the bench's op families and these disagree)."""
    bad = sorted({_short(n)[:80] for n in names if _short(n).startswith('conv_') and family(n)[0] not in CONV_FAMILIES})
    if bad:
        raise SystemExit('rocprof_families: conv kernels missing from the family table: %s' % bad)


def _find(d, suffix):
    hits = sorted(glob.glob(os.path.join(d, '**', '*' + suffix), recursive=True))
    if not hits:
        raise FileNotFoundError('no *%s under %s' % (suffix, d))
    return hits


def _rows(d):
    rows = []
    for path in _find(d, 'kernel_trace.csv'):
        with open(path) as f:
            rows += [(r['Kernel_Name'], int(r['Start_Timestamp']), int(r['End_Timestamp'])) for r in csv.DictReader(f)]
    return sorted(rows, key=lambda r: r[1])


def windows(rows):
    """Consecutive pairs of marker dispatches -> [(lo, hi), ...] in time order:
    bench.py stamps the timed region (graph replays) and then its eager
    timing pass; a kernel is inside a window when it starts after the opening
    marker ends and ends before the closing marker starts."""
    m = [(s, e) for n, s, e in rows if MARKER in n]
    return [(m[i][1], m[i + 1][0]) for i in range(0, len(m) - 1, 2)]


def kernel_trace(rows, window=None):
    fams = defaultdict(lambda: {'calls': 0, 'dispatches': 0, 'ns': 0})
    for name, t0, t1 in rows:
        if MARKER in name or (window and not (t0 >= window[0] and t1 <= window[1])):
            continue
        fam, prim = family(name)
        o = fams[fam]
        o['dispatches'] += 1
        o['calls'] += int(prim)
        o['ns'] += t1 - t0
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


def _pmc_rows(d, counter):
    rows = []
    for path in _find(d, 'counter_collection.csv'):
        with open(path) as f:
            for r in csv.DictReader(f):
                if r['Counter_Name'] == counter:
                    rows.append((int(r['Dispatch_Id']), r['Kernel_Name'], float(r['Counter_Value']),
                                 int(r['Start_Timestamp']), int(r['End_Timestamp'])))
    return sorted(rows)


def per_op(d, counter, ops):
    """The counter summed per conv op of bench.py's timing pass (its ops in
    issue order from --op-log): the pass lies between the 3rd and 4th marker;
    on one stream its dispatches come in issue order, each op's primary
    kernel opening it and its secondaries (split-K reduce) following."""
    rows = _pmc_rows(d, counter)
    m = [(s, e) for _, n, _, s, e in rows if MARKER in n]
    if len(m) < 4:
        raise SystemExit('rocprof_families: %s has no timing-pass markers (run bench.py with the timer)' % d)
    lo, hi = m[2][1], m[3][0]
    conv = iter([i for i, o in enumerate(ops) if o[0] in CONV_FAMILIES])
    vals, cur = [0.0] * len(ops), None
    for _, name, v, s, e in rows:
        if s < lo or e > hi or MARKER in name:
            continue
        fam, prim = family(name)
        if fam not in CONV_FAMILIES:
            continue
        if prim:
            cur = next(conv)
            if ops[cur][0] != fam:
                raise SystemExit('rocprof_families: op %d is %s, its dispatch %s' % (cur, ops[cur][0], name[:60]))
        vals[cur] += v
    if next(conv, None) is not None:
        raise SystemExit('rocprof_families: fewer conv dispatches than ops in the timing pass')
    return vals


def op_table(fetch_dir, write_dir, op_log):
    """Per conv shape and direction: PMC HBM bytes per call (FETCH_SIZE x 2 +
    WRITE_SIZE) against its algorithmic bytes, and the excess per step."""
    with open(op_log) as f:
        meta = json.load(f)
    ops = meta['ops']
    rd, wr = per_op(fetch_dir, 'FETCH_SIZE', ops), per_op(write_dir, 'WRITE_SIZE', ops)
    groups = defaultdict(lambda: [0, 0.0, 0.0, 0.0])
    for i, (kind, key, fl, nb, nd) in enumerate(ops):
        if kind not in CONV_FAMILIES:
            continue
        g = groups[(kind, key)]
        g[0] += 1
        g[1] += nb
        g[2] += 2.0 * rd[i] * 1024 + wr[i] * 1024
        g[3] += fl
    per = meta.get('timing_steps', 1)
    out = []
    for (kind, key), (n, nb, pb, fl) in groups.items():
        out.append({'kind': kind, 'shape': key, 'calls_per_step': n / per,
                    'algorithmic_bytes_per_call': round(nb / n), 'pmc_bytes_per_call': round(pb / n),
                    'pmc_over_algorithmic': round(pb / nb, 3) if nb else None,
                    'excess_MB_per_step': round((pb - nb) / per / 1e6, 2),
                    'gflop_per_call': round(fl / n / 1e9, 3)})
    out.sort(key=lambda r: -r['excess_MB_per_step'])
    tot = {k: [0.0, 0.0] for k in CONV_FAMILIES}
    for r in out:
        tot[r['kind']][0] += r['algorithmic_bytes_per_call'] * r['calls_per_step']
        tot[r['kind']][1] += r['pmc_bytes_per_call'] * r['calls_per_step']
    fam = {k: {'algorithmic_MB_per_step': round(a / 1e6, 1), 'pmc_MB_per_step': round(p / 1e6, 1),
               'pmc_over_algorithmic': round(p / a, 3) if a else None} for k, (a, p) in tot.items()}
    return out, fam


def _bench_line(path):
    """The JSON line bench.py printed in the traced run (its log file)."""
    with open(path) as f:
        for line in f:
            if line.startswith('{') and '"metric"' in line:
                return json.loads(line)
    raise SystemExit('rocprof_families: no bench line in %s' % path)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--trace', required=True)
    ap.add_argument('--fetch')
    ap.add_argument('--write')
    ap.add_argument('--mfma')
    ap.add_argument('--steps', type=int, default=0, help='steps in the traced run (warmup+timed) for per-step totals')
    ap.add_argument('--bench-line', help='log of the traced bench.py run: its line gives the algorithmic FLOPs / bytes '
                                         'per call of each conv family and the number of timed steps')
    ap.add_argument('--ops', help='op log of the PMC runs (bench.py --op-log): adds the per-shape PMC table')
    ap.add_argument('--out')
    ap.add_argument('--config', default='C2', help='bench.py workload the runs were taken on')
    a = ap.parse_args()
    rows = _rows(a.trace)
    check_complete(n for n, _, _ in rows)
    wins = windows(rows)
    line = _bench_line(a.bench_line) if a.bench_line else None
    fams = kernel_trace(rows, wins[0] if wins else None)
    fetch = pmc(a.fetch, 'FETCH_SIZE') if a.fetch else None
    write = pmc(a.write, 'WRITE_SIZE') if a.write else None
    busy = pmc(a.mfma, 'SQ_VALU_MFMA_BUSY_CYCLES') if a.mfma else None
    gui = pmc(a.mfma, 'GRBM_GUI_ACTIVE') if a.mfma else None
    if wins and line:
        a.steps = line['steps']          # the window holds exactly the K timed replays
    elif a.steps <= 0:   # counted: one adam_tick_kernel per optimizer step, 7 per C2 train step
        ticks = fams.get('adam_tick_kernel', {}).get('calls', 0)
        a.steps = round(ticks / 7) if ticks else 0
    alg = (line or {}).get('roofline', {}).get('families', {})
    out = {}
    for fam, o in sorted(fams.items(), key=lambda kv: -kv[1]['ns']):
        calls = max(o['calls'], 1)
        e = {'calls': o['calls'], 'dispatches': o['dispatches'], 'total_ms': round(o['ns'] * 1e-6, 6),
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
        if a.steps:
            e['ms_per_step'] = round(e['total_ms'] / a.steps, 6)
            e['calls_per_step'] = round(o['calls'] / a.steps, 2)
        q = alg.get(fam)
        if q and q.get('algorithmic_flops_per_launch') and a.steps:
            # the bench's own per-call algorithmic figures (same op families, same config)
            e['algorithmic_flops_per_call'] = q['algorithmic_flops_per_launch']
            e['algorithmic_bytes_per_call'] = q['algorithmic_bytes_per_launch']
            e['bench_launches_per_step'] = q['launches_per_step']
            sec = e['total_ms'] * 1e-3 / a.steps
            e['frac_in_step'] = round(e['algorithmic_flops_per_call'] * e['calls_per_step'] / sec / MFMA_PEAK, 4)
            e['algorithmic_hbm_frac_in_step'] = round(
                e['algorithmic_bytes_per_call'] * e['calls_per_step'] / sec / HBM_PEAK, 4)
            if e.get('hbm_bytes_per_call'):
                e['pmc_over_algorithmic'] = round(e['hbm_bytes_per_call'] / e['algorithmic_bytes_per_call'], 3)
        out[fam] = e
    total_ns = sum(o['ns'] for o in fams.values())
    res = {'families': out, 'gpu_busy_ms_total': round(total_ns * 1e-6, 3), 'config': a.config,
           'window': 'the timed graph replays between bench.py\'s markers' if wins else 'the whole trace'}
    res.update(_provenance())
    if a.steps:
        res['steps'] = a.steps
        res['gpu_busy_ms_per_step'] = round(total_ns * 1e-6 / a.steps, 3)
        cp = [out.get(f, {}) for f in CONV_FAMILIES]
        if all('algorithmic_bytes_per_call' in f for f in cp):
            ab = sum(f['algorithmic_bytes_per_call'] * f['calls_per_step'] for f in cp)
            ms = sum(f['ms_per_step'] for f in cp)
            res['conv_path'] = {'algorithmic_bytes_per_step': round(ab), 'kernel_ms_per_step': round(ms, 4),
                                'algorithmic_hbm_frac': round(ab / (ms * 1e-3) / HBM_PEAK, 4)}
            if all('hbm_bytes_per_call' in f for f in cp):
                pb = sum(f['hbm_bytes_per_call'] * f['calls_per_step'] for f in cp)
                res['conv_path']['pmc_bytes_per_step'] = round(pb)
                res['conv_path']['pmc_hbm_frac'] = round(pb / (ms * 1e-3) / HBM_PEAK, 4)
    if len(wins) > 1:   # bench.py's eager, single-stream timing pass: what its HIP events time
        tp = kernel_trace(rows, wins[1])
        res['timing_pass'] = {f: {'calls': tp[f]['calls'], 'total_ms': round(tp[f]['ns'] * 1e-6, 6),
                                  'avg_call_us': round(tp[f]['ns'] / max(tp[f]['calls'], 1) * 1e-3, 2)}
                              for f in CONV_FAMILIES if f in tp}
    if a.ops and a.fetch and a.write:
        res['per_shape'], res['per_shape_families'] = op_table(a.fetch, a.write, a.ops)
    txt = json.dumps(res, indent=1)
    if a.out:
        with open(a.out, 'w') as f:
            f.write(txt + '\n')
    print(txt)


if __name__ == '__main__':
    main()
