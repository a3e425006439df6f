#!/bin/bash
# Round evidence for one build, in the order the bench line needs it:
#   1. all -m gpu tests (parity log),
#   2. the rocprofv3 kernel trace + PMC passes (gpu_profile.sh), copied into
#      profiles/<TAG>_C2_families.json on the box so that
#   3. the C2 bench line (20 steps) quotes the profile of this same build
#      (traffic_matches_this_build, frac_in_step),
#   4. the replayed step's phase stamps, 5. the C3 line.
# Copy gpurun_out/<TAG>_* and gpurun_out/prof_<TAG>/ into profiles/ afterwards.
TAG=${1:-r06final}
source ./run_gpu_steps.sh
export EEGAN_PARITY_LOG=gpurun_out/${TAG}_parity_log.txt
step 700 ${TAG}_gputests python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
bash tools/gpu_profile.sh $TAG || exit $?
cp gpurun_out/prof_$TAG/families.json profiles/${TAG}_C2_families.json || exit 1
step 400 ${TAG}_bench python3 bench.py --steps 20 --warmup 5
grep -h '"metric"' gpurun_out/${TAG}_bench.log | cut -c1-300
step 300 ${TAG}_phases python3 -u tools/stamp_phases.py
step 400 ${TAG}_bench_C3 python3 bench.py --config C3 --steps 10 --warmup 3 --no-cpu-baseline
grep -h '"metric"' gpurun_out/${TAG}_bench_C3.log | cut -c1-200
