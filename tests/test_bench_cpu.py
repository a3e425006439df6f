"""bench.py's measurement plumbing on the CPU: `python bench.py --gpus N`
without a launcher starts an N-rank torch.distributed.run child job (one rank
per GPU, port bound by the store itself) and relays only rank 0's JSON line;
a rank whose job size differs from --gpus refuses to report."""
import json
import os
import subprocess
import sys

from _util import REPO

sys.path.insert(0, REPO)
import bench  # noqa: E402


def test_launcher_argv():
    argv = bench.launcher_argv(8, ['--gpus', '8', '--steps', '20', '--warmup', '5'])
    assert argv[:3] == [sys.executable, '-m', 'torch.distributed.run']
    assert '--standalone' in argv and argv[argv.index('--local-addr') + 1] == '127.0.0.1'
    assert argv[argv.index('--nproc-per-node') + 1] == '8'
    assert '--master-port' not in argv
    i = argv.index(os.path.join(REPO, 'bench.py'))
    assert argv[i + 1:] == ['--gpus', '8', '--steps', '20', '--warmup', '5']


def test_launch_ranks_relays_rank0_line(tmp_path, monkeypatch, capsys):
    script = tmp_path / 'fake_ranks.py'
    script.write_text('import json, sys\n'
                      'print("some rank chatter")\n'
                      'print(json.dumps({"metric": "m", "value": 1.5, "n_gpus": 2}))\n'
                      'sys.exit(int(sys.argv[1]))\n')
    monkeypatch.setattr(bench, 'launcher_argv', lambda n, argv: [sys.executable, str(script)] + list(argv))
    assert bench.launch_ranks(2, ['0']) == 0
    out, err = capsys.readouterr()
    assert [json.loads(x) for x in out.splitlines()] == [{'metric': 'm', 'value': 1.5, 'n_gpus': 2}]
    assert 'some rank chatter' in err
    assert bench.launch_ranks(2, ['3']) == 3           # the job's status is the launcher's


def test_rank_refuses_mismatched_world(tmp_path):
    """A rank started with --gpus 2 in a one-rank job (WORLD_SIZE=1) must not
    print a line for the wrong GPU count."""
    env = dict(os.environ, WORLD_SIZE='1', RANK='0', LOCAL_RANK='0', EEGAN_DIST_BACKEND='gloo')
    r = subprocess.run([sys.executable, os.path.join(REPO, 'bench.py'), '--gpus', '2', '--steps', '1'],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert 'refusing to report' in r.stderr
    assert not any(l.startswith('{') for l in r.stdout.splitlines())
