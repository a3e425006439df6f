#!/bin/bash
# in-process A/B: fused split-K finish, resident-weight halo kernel
source ./run_gpu_steps.sh
TAG=${1:-r05af}
step 600 ${TAG}_ab python3 -u tools/ab_inproc.py "EEGAN_CONV=" "EEGAN_CONV=splitk_fused=0" "EEGAN_CONV=halo_r=0" --reps 4 --steps 20
tail -8 gpurun_out/${TAG}_ab.log
