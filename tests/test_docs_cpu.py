"""INTEGRATION.md's environment-switch table against the code: every EEGAN_*
variable the package, the kernels' knob readers or bench.py read is listed,
and the count in the table's heading is the number of names in it."""
import os
import re

from _util import REPO

PKG = os.path.join(REPO, 'ee-gan_amd')


def _read_vars():
    found = set()
    pat = re.compile(r'''(?:environ\.get\(|environ\[|getenv\()\s*['"](EEGAN_[A-Z0-9_]+)['"]''')
    files = [os.path.join(REPO, 'bench.py')]
    for sub in ('eegan_hip', 'csrc', ''):
        d = os.path.join(PKG, sub)
        files += [os.path.join(d, f) for f in os.listdir(d)
                  if f.endswith(('.py', '.hip', '.cpp', '.h')) and os.path.isfile(os.path.join(d, f))]
    for f in files:
        with open(f) as fh:
            found |= set(pat.findall(fh.read()))
    return found


def test_switch_table_lists_every_variable_read():
    with open(os.path.join(REPO, 'INTEGRATION.md')) as fh:
        doc = fh.read()
    start = doc.index('Environment switches (')
    end = doc.index('Measured negatives are not kept as switches')
    table = set(re.findall(r'`(EEGAN_[A-Z0-9_]+)`', doc[start:end]))
    missing = _read_vars() - table
    assert not missing, sorted(missing)
    count = int(re.match(r'Environment switches \((\d+);', doc[start:]).group(1))
    assert count == len(table)
