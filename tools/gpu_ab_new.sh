#!/bin/bash
# In-process A/B of the round's new conv paths on the replayed step (base = all on)
source "$(dirname "$0")/../run_gpu_steps.sh"
cd "$GRAFT_REPO_ROOT"
step 600 ab python3 -u tools/ab_inproc.py "EEGAN_CONV_S2B=0 EEGAN_CONV_1X1=0 EEGAN_CONV_STAGE_EPI=0" "EEGAN_CONV_STAGE_EPI=0" "EEGAN_CONV_1X1=0" --reps 4 --steps 20
tail -4 gpurun_out/ab.log
