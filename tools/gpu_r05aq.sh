#!/bin/bash
source ./run_gpu_steps.sh
TAG=${1:-r05aq}
P=py:eegan_hip.trainer
step 900 ${TAG}_ab python3 -u tools/ab_inproc.py "$P.GEN_SIDE=False" "$P.LANE_ORDER='fwd'" "$P.GTERM_GRAD_EARLY=0" "$P.DAMSM_GRAD_EARLY=False" --reps 3 --steps 20
tail -5 gpurun_out/${TAG}_ab.log
