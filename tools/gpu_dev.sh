#!/bin/bash
# Development cycle on the GPU box: all -m gpu tests, the replayed step's
# phase timeline, a bench line.  Stops at the first crash / timeout.
source "$(dirname "$0")/../run_gpu_steps.sh"
cd "$GRAFT_REPO_ROOT"
TAG=${1:-dev}
step 600 gputests_$TAG python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step 300 phases_$TAG python3 -u tools/stamp_phases.py
step 400 bench_$TAG python3 bench.py --cpu-seconds 5
grep -h '"metric"' gpurun_out/bench_$TAG.log | cut -c1-600
