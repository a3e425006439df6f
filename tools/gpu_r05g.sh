#!/bin/bash
# run-to-run determinism of the eager C2 step: default, unfused split-K, one stream
source ./run_gpu_steps.sh
TAG=${1:-r05g}
step 300 ${TAG}_det python3 tools/determinism.py --config C2 --reps 5 --steps 2
step 300 ${TAG}_det_nofuse env EEGAN_CONV=splitk_fused=0 python3 tools/determinism.py --config C2 --reps 5 --steps 2
step 300 ${TAG}_det_1s python3 tools/determinism.py --config C2 --reps 5 --steps 2 --nostreams
grep -h "determinism" gpurun_out/${TAG}_det*.log
