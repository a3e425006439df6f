#!/bin/bash
# Diagnosis in one call: the rocprofv3 kernel trace + PMC passes of bench.py
# (gpu_profile.sh -> gpurun_out/prof_<TAG>/families.json, conv groups) and the
# whole step run eagerly on one stream with phase stamps under a kernel trace,
# grouped per phase and kernel (tools/lane_trace.py -> gpurun_out/<TAG>_lanes.txt).
TAG=${1:-diag}
source ./run_gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_profile.sh $TAG || exit $?
step 600 ${TAG}_lane_trace rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lane_$TAG -o run -- \
  python3 tools/lane_trace.py --d -1 --reps 2
LANE_TOP=25 python3 tools/lane_trace.py --report gpurun_out/lane_$TAG > gpurun_out/${TAG}_lanes.txt
find gpurun_out/lane_$TAG -name '*.csv' -size +20M -delete
