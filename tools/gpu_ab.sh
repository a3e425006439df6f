#!/bin/bash
# Quick GPU cycle after a kernel change: kernel + model parity, then the bench
# line and the per-dispatch group table of a short traced run.
source "$(dirname "$0")/../run_gpu_steps.sh"
cd "$GRAFT_REPO_ROOT"
step 600 gputests python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step 300 bench python3 bench.py --no-cpu-baseline
grep -h '"metric"' gpurun_out/bench.log
