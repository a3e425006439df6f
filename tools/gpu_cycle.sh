#!/bin/bash
# GPU cycle: every -m gpu test (parity log kept), the DAMSM microbench and
# the default bench line.  Stops at the first crash/timeout.
source "$(dirname "$0")/../run_gpu_steps.sh"
cd "$GRAFT_REPO_ROOT"
TAG=${1:-cycle}
export EEGAN_PARITY_LOG=gpurun_out/parity_$TAG.txt
rm -f "$EEGAN_PARITY_LOG"
step 900 gputests python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -s
step 300 damsm python3 tools/damsm_bench.py --out gpurun_out/damsm_$TAG.json
step 600 bench python3 bench.py --no-cpu-baseline
grep -h '"metric"' gpurun_out/bench.log
