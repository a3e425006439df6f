#!/bin/bash
# Idle time between kernels in graph replays: union of kernel intervals vs span.
source "$(dirname "$0")/../run_gpu_steps.sh"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step 300 gaps rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gaps -o run -- \
  python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-timer
python3 tools/trace_gaps.py gpurun_out/gaps > gpurun_out/gaps.txt
find gpurun_out/gaps -name '*.csv' -size +20M -delete
