#!/bin/bash
# in-process knob re-check on the post-fix step
source ./run_gpu_steps.sh
TAG=${1:-r05aj}
step 900 ${TAG}_ab python3 -u tools/ab_inproc.py "EEGAN_CONV=" "EEGAN_CONV=wgrad_target=1024" "EEGAN_CONV=target=1024" "EEGAN_CONV=halo_r_tpb=8" "EEGAN_CONV=halo_nb=1" --reps 3 --steps 20
tail -6 gpurun_out/${TAG}_ab.log
