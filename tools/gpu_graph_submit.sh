#!/bin/bash
# Host submission cost of the captured step graph under runtime settings
# (tools/probe/graph_submit.py, one process per setting).
source "$(dirname "$0")/../run_gpu_steps.sh"
cd "$GRAFT_REPO_ROOT"
step 300 gs_default python3 -u tools/probe/graph_submit.py ${GS_ARGS}
grep -h GRAPHSUBMIT gpurun_out/gs_*.log
