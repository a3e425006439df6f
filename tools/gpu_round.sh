#!/bin/bash
# Round evidence in one call: all -m gpu tests (parity log under gpurun_out/),
# the bench line, the replayed step's phase stamps, then the rocprofv3 kernel
# trace + PMC passes (gpu_profile.sh).  Stops at the first crash / timeout.
TAG=${1:-r06a}
source ./run_gpu_steps.sh
export EEGAN_PARITY_LOG=gpurun_out/${TAG}_parity_log.txt
step 1100 ${TAG}_gputests python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step 400 ${TAG}_bench python3 bench.py --steps 20 --warmup 5
grep -h '"metric"' gpurun_out/${TAG}_bench.log | cut -c1-400
[ "${PROFILE:-1}" = 1 ] || exit 0
step 300 ${TAG}_phases python3 -u tools/stamp_phases.py
bash tools/gpu_profile.sh $TAG
