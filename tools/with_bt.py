#!/usr/bin/env python
"""Run a Python script in THIS process with a native-backtrace crash handler
installed (tools/segv/segv_bt.c, built on first use):

    python tools/with_bt.py tools/stamp_phases.py [args...]
"""
import ctypes
import os
import runpy
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, 'segv', 'libsegvbt.so')
if not os.path.exists(SO):
    subprocess.check_call(['gcc', '-shared', '-fPIC', '-O1', '-o', SO, os.path.join(HERE, 'segv', 'segv_bt.c')])
ctypes.CDLL(SO).segv_bt_install()
sys.argv = sys.argv[1:]
runpy.run_path(sys.argv[0], run_name='__main__')
