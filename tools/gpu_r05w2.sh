#!/bin/bash
# phase stamps of the replayed step + rocprofv3 trace/PMC passes (gpu_profile.sh)
source ./run_gpu_steps.sh
TAG=${1:-r05w}
step 300 ${TAG}_phases python3 -u tools/stamp_phases.py
bash tools/gpu_profile.sh $TAG
