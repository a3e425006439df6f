"""tools/rocprof_families.py on synthetic rocprofv3 CSVs: the one kernel ->
family table covers every conv kernel (an unknown conv_ kernel is an error),
the families are summed over the timed replays between bench.py's markers
only, the in-step figures recompute from the written file, and the per-shape
PMC table matches dispatches to the op log in issue order."""
import csv
import json
import os
import subprocess
import sys

import pytest

from _util import REPO

sys.path.insert(0, os.path.join(REPO, 'tools'))
import rocprof_families as RF  # noqa: E402

NS = '(anonymous namespace)::'


@pytest.mark.parametrize('name,fam,prim', [
    ('void ' + NS + 'conv_fast_kernel<0, 64, 64, 2, 4, 2>(' + NS + 'ConvArgs, long, long)', 'conv_fwd', True),
    ('void ' + NS + 'conv_fast_kernel<1, 128, 64, 2, 4, 2>(' + NS + 'ConvArgs, long, long)', 'conv_bwd_data', True),
    ('void ' + NS + 'conv_halo3r_kernel<0>(' + NS + 'ConvArgs, long, long, int, int)', 'conv_fwd', True),
    ('void ' + NS + 'conv_halo3r_kernel<1>(' + NS + 'ConvArgs, long, long, int, int)', 'conv_bwd_data', True),
    ('void ' + NS + 'conv_halo3_kernel<1, 4, 4, false, 1>(' + NS + 'ConvArgs, long, long)', 'conv_bwd_data', True),
    (NS + 'conv_s2fwd_kernel(' + NS + 'ConvArgs, long)', 'conv_fwd', True),
    ('void ' + NS + 'conv_s2bwd_lds_kernel<1, 2>(' + NS + 'ConvArgs, int, int)', 'conv_bwd_data', True),
    ('void ' + NS + 'conv_thin_lds_kernel<1, 2, 9>(' + NS + 'ConvArgs, int, int)', 'conv_bwd_data', True),
    ('void ' + NS + 'conv_1x1_kernel<0, 4, 1, 1>(' + NS + 'ConvArgs, int, int)', 'conv_fwd', True),
    ('void ' + NS + 'conv_wgrad_halo3_kernel<64>(' + NS + 'WgradArgs, int, int, int)', 'conv_bwd_weight', True),
    ('void ' + NS + 'conv_wgrad_thin_kernel<2>(' + NS + 'WgradArgs, int, int, int)', 'conv_bwd_weight', True),
    ('void ' + NS + 'conv_wgrad_fast_kernel<128, 128, 2>(' + NS + 'WgradArgs, long, long, int, int)',
     'conv_bwd_weight', True),
    ('void ' + NS + 'conv_splitk_reduce_kernel<0>(' + NS + 'ConvArgs)', 'conv_fwd', False),
    ('void ' + NS + 'conv_splitk_reduce_kernel<1>(' + NS + 'ConvArgs)', 'conv_bwd_data', False),
    ('void ' + NS + 'wgrad_quad_reduce_kernel<256, 1>(float const*, int, long)', 'conv_bwd_weight', False),
    ('void colsum_rows_kernel<32, 8, float, float, ' + NS + 'WgradMap>(float const*)', 'conv_bwd_weight', False),
])
def test_family_table(name, fam, prim):
    assert RF.family(name) == (fam, prim)


def test_unknown_conv_kernel_is_an_error():
    with pytest.raises(SystemExit):
        RF.check_complete(['void ' + NS + 'conv_new_kernel<0>(' + NS + 'ConvArgs)'])
    RF.check_complete(['void ' + NS + 'bnmod_fwd_kernel<true>(x)'])


FWD = 'void ' + NS + 'conv_fast_kernel<0, 64, 64, 2, 4, 2>(' + NS + 'ConvArgs, long, long)'
RED = 'void ' + NS + 'conv_splitk_reduce_kernel<0>(' + NS + 'ConvArgs)'
WG = 'void ' + NS + 'conv_wgrad_fast_kernel<128, 128, 2>(' + NS + 'WgradArgs, long, long, int, int)'
MARK = NS + 'stamp_kernel(unsigned long long*)'
OTHER = 'void ' + NS + 'bnmod_fwd_kernel<true>(x)'


def _trace(path, rows):
    with open(path, 'w', newline='') as f:
        w = csv.writer(f)
        w.writerow(['Kernel_Name', 'Start_Timestamp', 'End_Timestamp'])
        for r in rows:
            w.writerow(r)


def _pmc(path, counter, rows):
    with open(path, 'w', newline='') as f:
        w = csv.writer(f)
        w.writerow(['Dispatch_Id', 'Kernel_Name', 'Counter_Name', 'Counter_Value', 'Start_Timestamp', 'End_Timestamp'])
        for i, (n, v, s, e) in enumerate(rows):
            w.writerow([i + 1, n, counter, v, s, e])


def test_windows_perstep_and_per_shape(tmp_path):
    tr = tmp_path / 'trace'
    tr.mkdir()
    # warm-up outside the window, 2 timed steps inside, then the timing pass (2nd window)
    rows = [(FWD, 0, 50), (MARK, 100, 101),
            (FWD, 110, 120), (RED, 121, 123), (WG, 130, 150), (OTHER, 151, 160),
            (FWD, 200, 210), (RED, 211, 213), (WG, 220, 240),
            (MARK, 300, 301), (MARK, 400, 401), (FWD, 410, 415), (RED, 416, 417), (WG, 420, 430), (MARK, 500, 501)]
    _trace(tr / 'run_kernel_trace.csv', rows)
    line = {'metric': 'm', 'steps': 2, 'roofline': {'families': {
        'conv_fwd': {'algorithmic_flops_per_launch': 1e9, 'algorithmic_bytes_per_launch': 1000, 'launches_per_step': 1},
        'conv_bwd_data': {'algorithmic_flops_per_launch': 1e9, 'algorithmic_bytes_per_launch': 1000,
                          'launches_per_step': 0},
        'conv_bwd_weight': {'algorithmic_flops_per_launch': 2e9, 'algorithmic_bytes_per_launch': 4000,
                            'launches_per_step': 1}}}}
    (tmp_path / 'bench.log').write_text('noise\n' + json.dumps(line) + '\n')
    # PMC runs: one eager step, then the timing pass with one fwd op and one wgrad op
    ops = {'config': 'C2', 'timing_steps': 1, 'ops': [['conv_fwd', 'N1 a', 1e9, 1000, 2], ['gemm_f32', 'g', 1, 1, 1],
                                                      ['conv_bwd_weight', 'N1 b', 2e9, 4000, 1]]}
    (tmp_path / 'ops.json').write_text(json.dumps(ops))
    for sub, counter, vals in (('fetch', 'FETCH_SIZE', (1.0, 0.25, 3.0)), ('write', 'WRITE_SIZE', (0.5, 0.5, 1.0))):
        d = tmp_path / sub
        d.mkdir()
        _pmc(d / 'run_counter_collection.csv', counter,
             [(MARK, 0, 0, 1), (FWD, 9.0, 2, 3), (MARK, 0, 4, 5), (MARK, 0, 6, 7),
              (FWD, vals[0], 8, 9), (RED, vals[1], 10, 11), (OTHER, 7.0, 12, 13), (WG, vals[2], 14, 15),
              (MARK, 0, 16, 17)])
    out = tmp_path / 'fam.json'
    subprocess.run([sys.executable, os.path.join(REPO, 'tools', 'rocprof_families.py'), '--trace', str(tr),
                    '--fetch', str(tmp_path / 'fetch'), '--write', str(tmp_path / 'write'),
                    '--bench-line', str(tmp_path / 'bench.log'), '--ops', str(tmp_path / 'ops.json'),
                    '--out', str(out)], check=True, capture_output=True)
    res = json.loads(out.read_text())
    f = res['families']['conv_fwd']
    assert res['steps'] == 2 and f['calls'] == 2 and f['dispatches'] == 4   # warm-up and timing pass excluded
    assert f['total_ms'] == pytest.approx((10 + 2 + 10 + 2) * 1e-6)
    assert f['calls_per_step'] == 1.0
    # frac_in_step recomputes from the file: algorithmic FLOPs per step / in-step seconds / peak
    sec = f['total_ms'] * 1e-3 / res['steps']
    assert f['frac_in_step'] == pytest.approx(round(1e9 * f['calls_per_step'] / sec / 2.5e15, 4))
    assert res['timing_pass']['conv_fwd'] == {'calls': 1, 'total_ms': 6e-6, 'avg_call_us': 0.01}
    ps = {r['shape']: r for r in res['per_shape']}
    # fwd op: its conv kernel + reduce; FETCH x2 + WRITE, KB -> bytes
    assert ps['N1 a']['pmc_bytes_per_call'] == round((2 * (1.0 + 0.25) + (0.5 + 0.5)) * 1024)
    assert ps['N1 b']['pmc_bytes_per_call'] == round((2 * 3.0 + 1.0) * 1024)
    assert ps['N1 b']['pmc_over_algorithmic'] == round(7 * 1024 / 4000, 3)
