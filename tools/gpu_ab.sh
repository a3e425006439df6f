#!/bin/bash
# Quick GPU cycle after a kernel change: kernel + model parity, then the bench
# line and the per-dispatch group table of a short traced run.
source "$(dirname "$0")/../run_gpu_steps.sh"
cd "$GRAFT_REPO_ROOT"
step 600 gputests python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step 300 bench python3 bench.py --no-cpu-baseline
grep -h '"metric"' gpurun_out/bench.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step 300 trace rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ab_trace -o run -- \
  python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-timer
python3 tools/dispatch_groups.py gpurun_out/ab_trace --steps 6 --top 40 > gpurun_out/ab_groups.txt
python3 tools/dispatch_groups.py gpurun_out/ab_trace --steps 6 --top 60 --by-name > gpurun_out/ab_names.txt
find gpurun_out/ab_trace -name '*.csv' -delete
