#!/bin/bash
# in-process sweep of the conv planner knobs not re-checked this round
source ./run_gpu_steps.sh
TAG=${1:-r05bb}
step 900 ${TAG}_ab python3 -u tools/ab_inproc.py "EEGAN_CONV=1x1_blocks=512" "EEGAN_CONV=1x1_blocks=2048" \
  "EEGAN_CONV=s2b_blocks=256" "EEGAN_CONV=s2b_blocks=1024" "EEGAN_CONV=wgrad_minp=256" "EEGAN_CONV=wgrad_minp=1024" \
  "EEGAN_CONV=wgrad_quad_mink=512" "EEGAN_CONV=wgrad_quad_mink=2048" "EEGAN_CONV=wgrad_target=256" \
  "EEGAN_CONV=halo_r_tpb=4" "EEGAN_CONV=wgrad_stage_epi=1" --reps 3 --steps 20
tail -13 gpurun_out/${TAG}_ab.log
