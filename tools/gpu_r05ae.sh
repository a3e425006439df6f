#!/bin/bash
# halo3r default tile count + whole-step lane trace (one stream) for the generator phases
source ./run_gpu_steps.sh
TAG=${1:-r05ae}
step 300 ${TAG}_cb python3 tools/conv_bench.py --shapes d256_b0_3x3,c3x3_64_128 --dirs fwd,bwdd
grep -E "TF/s" gpurun_out/${TAG}_cb.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step 300 lt_all rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lt_all -o run -- python3 tools/lane_trace.py --d -1
LANE_TOP=40 python3 tools/lane_trace.py --report gpurun_out/lt_all > gpurun_out/${TAG}_lt_all_report.txt
find gpurun_out/lt_all -name '*.csv' -delete
