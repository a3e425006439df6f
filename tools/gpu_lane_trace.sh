#!/bin/bash
# Kernel-level phase breakdown: D256's d_update and the whole step (one stream), rocprofv3 kernel trace.
source "$(dirname "$0")/../run_gpu_steps.sh"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step 300 lt_d2 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lt_d2 -o run -- python3 tools/lane_trace.py --d 2
LANE_TOP=22 python3 tools/lane_trace.py --report gpurun_out/lt_d2 > gpurun_out/lt_d2_report.txt
step 300 lt_all rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lt_all -o run -- python3 tools/lane_trace.py --d -1
LANE_TOP=22 python3 tools/lane_trace.py --report gpurun_out/lt_all > gpurun_out/lt_all_report.txt
find gpurun_out/lt_d2 gpurun_out/lt_all -name '*.csv' -delete
