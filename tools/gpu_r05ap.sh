#!/bin/bash
source ./run_gpu_steps.sh
TAG=${1:-r05ap}
step 900 ${TAG}_ab python3 -u tools/ab_inproc.py "EEGAN_CONV=target=256" "EEGAN_CONV=mink=32" "EEGAN_CONV=mink=64" "EEGAN_CONV=target=384" --reps 3 --steps 20
tail -5 gpurun_out/${TAG}_ab.log
