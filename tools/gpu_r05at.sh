#!/bin/bash
# HEAD: all -m gpu tests + smoke
source ./run_gpu_steps.sh
TAG=${1:-r05at}
step 1000 ${TAG}_gputests python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
tail -2 gpurun_out/${TAG}_gputests.log
step 300 ${TAG}_smoke python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
tail -2 gpurun_out/${TAG}_smoke.log
