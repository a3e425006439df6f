#!/bin/bash
# HEAD at round end: all -m gpu tests, smoke, the default bench line
source ./run_gpu_steps.sh
TAG=${1:-r05ba}
step 1000 ${TAG}_gputests python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
tail -2 gpurun_out/${TAG}_gputests.log
step 300 ${TAG}_smoke python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
tail -2 gpurun_out/${TAG}_smoke.log
step 600 ${TAG}_bench python3 bench.py
tail -1 gpurun_out/${TAG}_bench.log
