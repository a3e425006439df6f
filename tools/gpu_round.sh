#!/bin/bash
# Round evidence in one call: device probe + all -m gpu tests with the parity
# log + bench line (gpu_r04a.sh), the replayed step's phase stamps, then the
# rocprofv3 kernel trace + PMC passes (gpu_profile.sh).
TAG=${1:-r04b}
bash tools/gpu_r04a.sh $TAG || exit $?
source ./run_gpu_steps.sh
step 300 ${TAG}_phases python3 -u tools/stamp_phases.py
bash tools/gpu_profile.sh $TAG
