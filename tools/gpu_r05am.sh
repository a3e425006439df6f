#!/bin/bash
source ./run_gpu_steps.sh
TAG=${1:-r05am}
step 600 ${TAG}_ab python3 -u tools/ab_inproc.py "EEGAN_CONV=wgrad_halo=0" "EEGAN_CONV=wgrad_halo_blocks=256" --reps 4 --steps 20
tail -4 gpurun_out/${TAG}_ab.log
