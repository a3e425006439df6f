#!/bin/bash
# Round-end style GPU cycle: all -m gpu tests, smoke(), bench with cpu_baseline.
source "$(dirname "$0")/../run_gpu_steps.sh"
cd "$GRAFT_REPO_ROOT"
step 900 gputests python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step 300 smoke python3 -c "import __graft_entry__ as g; g.smoke()"
step 600 bench python3 bench.py
grep -h '"metric"' gpurun_out/bench.log
