#!/usr/bin/env python
"""Per-kernel register / spill / LDS summary of one HIP source (hipcc
-Rpass-analysis=kernel-resource-usage), filtered by a name substring.

    python tools/kres.py ee-gan_amd/csrc/conv.hip conv_fast_kernel
"""
import re
import subprocess
import sys

src, pat = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else '')
out = subprocess.run(['/opt/rocm/bin/hipcc', '-O3', '-std=c++17', '-fPIC', '--offload-arch=gfx950', '-c', src, '-o',
                      '/tmp/_kres.o', '-Rpass-analysis=kernel-resource-usage'], capture_output=True, text=True).stderr
cur = None
rows = []
for line in out.splitlines():
    m = re.search(r'remark: (?:\s*)(Function Name|VGPRs|AGPRs|SGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|'
                  r'VGPRs Spill|SGPRs Spill|LDS Size \[bytes/block\]): (\S+)', line)
    if not m:
        continue
    k, v = m.group(1), m.group(2)
    if k == 'Function Name':
        cur = {'name': v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for r in rows:
    if pat in r['name']:
        n = subprocess.run(['c++filt', r['name']], capture_output=True, text=True).stdout.strip()
        print('%-72s vgpr %4s agpr %3s spill %3s scratch %4s lds %6s occ %s' % (
            n.replace('(anonymous namespace)::', '')[:72], r.get('VGPRs'), r.get('AGPRs'), r.get('VGPRs Spill'),
            r.get('ScratchSize [bytes/lane]'), r.get('LDS Size [bytes/block]'), r.get('Occupancy [waves/SIMD]')))
